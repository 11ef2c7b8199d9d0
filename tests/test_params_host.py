"""Variable inventory of U_NET (model/u_net.py) and host logic: names, Keras layouts, counts,
initializers, the flat HBM layout, the builder's ValueError, callbacks."""
import math
import os

import numpy as np
import pytest

from unet_amd.params import (ALIGN, check_input_size, compute_fans, count_params, flat_layout, init_weights,
                             unet_variables)


def test_counts_match_reference_topology():
    specs = unet_variables()
    tr, nt = count_params(specs)
    assert tr == 5_988_252 and nt == 11_776 and tr + nt == 6_000_028
    assert sum(s.trainable for s in specs) == 82 and len(specs) == 118
    specs21 = unet_variables(3, 21)
    assert count_params(specs21)[0] == 5_988_252 + 64 * 20 + 20


def test_keras_names_and_layouts():
    s = {v.name: v for v in unet_variables()}
    assert s["enc1_block1_sepconv/depthwise_kernel"].shape == (3, 3, 3, 1)
    assert s["enc1_block1_sepconv/pointwise_kernel"].shape == (1, 1, 3, 64)
    assert s["bneck_block2_sepconv/pointwise_kernel"].shape == (1, 1, 1024, 1024)
    assert s["dec4_upsample/kernel"].shape == (2, 2, 512, 1024)
    assert s["dec4_block1_sepconv/depthwise_kernel"].shape == (3, 3, 1024, 1)
    assert s["dec1_upsample/kernel"].shape == (2, 2, 64, 128)
    assert s["output_mask/kernel"].shape == (1, 1, 64, 1)
    assert not s["enc3_block2_bn/moving_variance"].trainable
    names = [v.name for v in unet_variables()]
    # Keras creation order: encoder, bottleneck, decoder (upsample before its blocks), head
    assert names.index("enc4_block2_bn/beta") < names.index("bneck_block1_sepconv/depthwise_kernel")
    assert names.index("dec4_upsample/bias") < names.index("dec4_block1_sepconv/depthwise_kernel")
    assert names[-2:] == ["output_mask/kernel", "output_mask/bias"]


def test_no_batchnorm_variant_has_biases():
    s = {v.name for v in unet_variables(use_batch_norm=False)}
    assert "enc1_block1_sepconv/bias" in s and not any("_bn/" in n for n in s)


def test_glorot_initializer():
    assert compute_fans((3, 3, 64, 1)) == (576, 9)
    assert compute_fans((1, 1, 64, 128)) == (64, 128)
    assert compute_fans((2, 2, 512, 1024)) == (2048, 4096)
    specs = unet_variables()
    w = init_weights(specs, 2301)
    k = w["enc2_block1_sepconv/pointwise_kernel"]
    lim = math.sqrt(6 / (64 + 128))
    assert np.abs(k).max() <= lim and np.abs(k).max() > 0.95 * lim
    assert abs(k.mean()) < 0.05 * lim
    assert np.all(w["enc1_block1_bn/gamma"] == 1) and np.all(w["enc1_block1_bn/moving_variance"] == 1)
    w2 = init_weights(specs, 2301)
    assert all(np.array_equal(w[n], w2[n]) for n in w)  # deterministic, portable


def test_flat_layout_alignment():
    specs = unet_variables()
    lay = flat_layout(specs, True)
    offs = sorted(lay.offsets.values())
    assert all(o % ALIGN == 0 for o in offs)
    assert lay.total >= 5_988_252 and lay.total - 5_988_252 < 82 * ALIGN


def test_input_size_validation():
    with pytest.raises(ValueError, match="tuple of"):
        check_input_size((256, 256))
    with pytest.raises(ValueError, match="divisible"):
        check_input_size((250, 256, 3))
    assert check_input_size((128, 128, 3)) == (128, 128, 3)


def test_builder_signature_mirrors_reference():
    import inspect
    from model.u_net import U_NET, conv_block, unet
    sig = inspect.signature(U_NET)
    assert list(sig.parameters)[:4] == ["input_size", "num_classes", "dropout_rate", "use_batch_norm"]
    assert sig.parameters["num_classes"].default == 1 and sig.parameters["dropout_rate"].default == 0.2
    assert list(inspect.signature(conv_block).parameters)[:5] == ["input_tensor", "num_filters", "kernel_size",
                                                                  "use_batch_norm", "name_prefix"]
    assert list(inspect.signature(unet).parameters)[:2] == ["input_size", "num_classes"]
    with pytest.raises(ValueError):
        U_NET((256, 256))


def test_callbacks_semantics():
    from unet_amd.callbacks import EarlyStopping, ReduceLROnPlateau

    class Opt:
        learning_rate = 1e-3

    class M:
        optimizer = Opt()
        stop_training = False
        w = [np.zeros(1)]

        def get_weights(self):
            return [x.copy() for x in self.w]

        def set_weights(self, w):
            self.w = w

    m = M()
    rl = ReduceLROnPlateau("val_mean_io_u", factor=0.2, patience=3, mode="max", min_lr=1e-6)
    rl.set_model(m)
    for e, v in enumerate([0.5, 0.6, 0.6, 0.6, 0.6]):
        rl.on_epoch_end(e, {"val_mean_io_u": v})
    assert abs(m.optimizer.learning_rate - 2e-4) < 1e-12
    es = EarlyStopping("val_mean_io_u", patience=2, mode="max", restore_best_weights=True)
    es.set_model(m)
    es.on_train_begin()
    for e, v in enumerate([0.5, 0.7, 0.6, 0.6]):
        m.w = [np.full(1, float(e))]
        es.on_epoch_end(e, {"val_mean_io_u": v})
    assert m.stop_training and m.w[0][0] == 1.0 and es.stopped_epoch == 3
    # the report scripts/train.py prints after fit (reference scripts/train.py:317-331)
    from scripts.train import training_summary

    class H:
        history = {"val_mean_io_u": [0.5, 0.7, 0.6, 0.6]}
    assert training_summary(H(), es, "val_mean_io_u", "max", 30) == [
        "Early stopping triggered at epoch 4",
        "Best monitored score (val_mean_io_u): 0.7000 (from epoch 2)"]  # 4 - patience 2
    es2 = EarlyStopping("val_mean_io_u", patience=10, mode="max")
    es2.on_train_begin()
    assert training_summary(H(), es2, "val_mean_io_u", "max", 4) == [
        "Best monitored score (val_mean_io_u): 0.7000 (from epoch 2)"]
    assert training_summary(H(), es2, "val_loss", "min", 4) == [
        "Best monitored score (val_loss): inf (from epoch N/A)"]


def test_train_sample_count_fallback(tmp_path, capsys):
    """scripts/train.py counts samples from the loaders, else lists the frame directories, else
    exits 1 (reference scripts/train.py:237-249)."""
    from scripts.train import TRAIN_FRAMES_DIR, VAL_FRAMES_DIR, count_samples

    class Bad:
        @property
        def samples(self):
            raise RuntimeError("no count")
    for d, n in ((TRAIN_FRAMES_DIR, 3), (VAL_FRAMES_DIR, 2)):
        os.makedirs(tmp_path / d)
        for i in range(n):
            (tmp_path / d / f"{i}.png").write_bytes(b"")
    assert count_samples(Bad(), Bad(), str(tmp_path)) == (3, 2)
    assert "(Fallback) Counted 3 train files, 2 val files." in capsys.readouterr().out
    with pytest.raises(SystemExit) as e:
        count_samples(Bad(), Bad(), str(tmp_path / "missing"))
    assert e.value.code == 1


def test_train_loader_error_banner(tmp_path, capsys):
    """A missing dataset tree ends train.py the reference's way: the 'Error initializing
    ImageDataGenerator' block closed by its dashed line, exit 1 (reference scripts/train.py:208-217).
    No device work happens before the loaders are built."""
    from scripts.train import main
    with pytest.raises(SystemExit) as e:
        main(["--dataset-root", str(tmp_path / "missing"), "--epochs", "1"])
    out = capsys.readouterr().out
    assert e.value.code == 1
    assert "\n--- Error initializing ImageDataGenerator ---\n" in out
    assert "-------------------------------------------\n" in out


def test_train_stdout_strings_match_reference():
    """The banner strings train.py prints around the training loop (reference
    scripts/train.py:301, 333-338): the TensorBoard log line and the closing dashed line of the
    training-error block."""
    import inspect
    import scripts.train as T
    src = inspect.getsource(T.main)
    assert 'TensorBoard logs will be saved to: {log_dir}' in src
    i = src.index('print("\\n--- Error during model training ---")')
    assert 'print("-----------------------------------\\n")' in src[i:]
