"""Inference through a captured HIP graph (UNetEngine.graph_predict, round 6) against the eager
inference forward: the same kernels on the same buffers, so the probabilities must be bitwise
equal -- per input shape (one graph each), on repeated replays, after the weights change under
the graph (a train step + AdamW: the graph reads weights, moving statistics and split planes
through their device pointers), and after release_buffers() (graphs dropped with the buffers).

Reference: model/u_net.py:55-112 (the forward), scripts/benchmark.py:254-260 (model.predict)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.mark.parametrize("size,ncls", [(64, 1), (128, 3)])
def test_graph_predict_equals_eager(size, ncls):
    from unet_amd.model import UNetModel
    from unet_amd.optim import AdamW

    rng = np.random.default_rng(size + ncls)
    model = UNetModel((size, size, 3), ncls, dropout_rate=0.2, device="cuda:0")
    eng = model.engine
    xs = {n: torch.as_tensor(rng.random((n, size, size, 3), dtype=np.float32), device="cuda:0") for n in (1, 3)}

    def both(x):
        eng.graph_predict = False
        e = eng.predict(x)
        eng.graph_predict = True
        g = eng.predict(x)
        return e, g

    for n, x in xs.items():
        e, g = both(x)
        assert torch.equal(e, g), n
        assert torch.equal(eng.predict(x), g)  # replay
    assert len(eng._pgraphs) == 2
    # weights change under the graphs: one train step (batch statistics, dropout, AdamW)
    model.compile(AdamW(learning_rate=1e-2, weight_decay=1e-4), "dice_loss")
    y = (rng.random((2, size, size, ncls)) > 0.5).astype(np.float32)
    before = eng.predict(xs[1]).clone()
    model.train_step(rng.random((2, size, size, 3), dtype=np.float32), y)
    for n, x in xs.items():
        e, g = both(x)
        assert torch.equal(e, g), n
    assert not torch.equal(before, eng.predict(xs[1]))
    assert len(eng._pgraphs) == 2  # no re-capture for a weight update
    eng.release_buffers()
    assert not eng._pgraphs
    e, g = both(xs[3])
    assert torch.equal(e, g)
    eng.graph_predict = False
