"""Multi-rank consistency check of the data-parallel train step (run under torch.distributed.run;
with UNET_DP_ONE_DEVICE=1 every rank shares GPU 0 and gloo carries the collectives).  Each rank
trains on its own synthetic shard; after the bucketed all-reduce every rank must hold bitwise the
same averaged gradients and the same post-AdamW weights (a bucket all-reduced before its
gradients were final, or never, shows up as a rank-dependent difference)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT]
import torch
import torch.distributed as dist

from bench import synthetic_batch
from unet_amd.dp import init_from_env
from unet_amd.model import UNetModel
from unet_amd.optim import AdamW

rank, world, local = init_from_env()
dev = torch.device("cuda", local)
torch.cuda.set_device(dev)
m = UNetModel((64, 64, 3), 1, dropout_rate=0.2, device=dev)
m.compile(AdamW(2e-3, 1e-4), "dice_loss")
m.enable_data_parallel(bucket_bytes=1 << 20)  # many buckets: exercises the held low-water mark
x, y = synthetic_batch(4, 64, 64, 1, 77 + rank, dev)
for _ in range(3):
    m.train_step(x, y)
torch.cuda.synchronize()
g = m.engine.grads.detach().clone().cpu()
p = m.engine.params.detach().clone().cpu()
gs = [torch.empty_like(g) for _ in range(world)]
ps = [torch.empty_like(p) for _ in range(world)]
dist.all_gather(gs, g)
dist.all_gather(ps, p)
ok = all(torch.equal(gs[0], t) for t in gs) and all(torch.equal(ps[0], t) for t in ps)
nz = float((g != 0).float().mean())
if rank == 0:
    print(f"dp_check world={world}: grads/params identical across ranks: {ok} (nonzero grad fraction {nz:.3f})")
dist.barrier()
dist.destroy_process_group()
sys.exit(0 if ok else 1)
