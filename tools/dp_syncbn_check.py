"""SyncBN correctness check (run under torch.distributed.run; with UNET_DP_ONE_DEVICE=1 every rank
shares GPU 0 and gloo carries the collectives).

Each rank trains one data-parallel step with SyncBN (model.enable_data_parallel(sync_bn=True):
every BatchNorm normalises over the GLOBAL batch -- forward records gathered and combined in rank
order, backward (sum g, sum g*xhat) all-reduced before dz is formed) on its shard of a global batch
of DP_CHECK_GLOBAL synthetic images (default 5 over 2 ranks: shards 3 + 2).  Dropout is off, so
the step must equal ONE single-process step on the whole global batch:
  * DP gradient (the all-reduced sum / world) == the full-batch gradient, relative L2 per tensor
    <= 2e-5 (fp32 reduction order: float sums all-reduced across replicas vs one replica's double
    chunk sums);
  * BN batch statistics -> moving mean / variance after the step == the full-batch model's,
    relative <= 1e-6, identical on every rank;
  * every rank holds bitwise identical gradients, weights and moving statistics.
Without SyncBN the same comparison fails by O(1e-2) (per-replica statistics), which the check
also prints (DP_CHECK_LOCAL=1 runs that variant).

DP_CHECK_DROP=1: dropout 0.2 with SyncBN.  Per-rank dropout salts rule out the
full-batch comparison, so the reference is the SAME two-rank SyncBN step (same seeds, same salts)
with the producers' fused BatchNorm-backward partials switched off (engine.fuse_bn_stats = False:
every block's (sum g, sum g*xhat) from a separate reduction over (da, z) with the mask applied
there), i.e. the dropout-masked partials of the Conv2DTranspose data gradient at the bottleneck
(bn_masked) are checked together with the SyncBN all-reduce: gradients within 1e-4, moving
statistics within 1e-6."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT]
import torch
import torch.distributed as dist

from bench import synthetic_batch
from unet_amd.dp import init_from_env, shard_bounds
from unet_amd.model import UNetModel
from unet_amd.optim import AdamW

rank, world, local = init_from_env()
dev = torch.device("cuda", local)
torch.cuda.set_device(dev)
G = int(os.environ.get("DP_CHECK_GLOBAL", "5"))
SYNC = os.environ.get("DP_CHECK_LOCAL") != "1"
DROP = 0.2 if os.environ.get("DP_CHECK_DROP") == "1" else 0.0
HW, SEED, LR, WD = 64, 5, 2e-3, 1e-4
x_all, y_all = synthetic_batch(G, HW, HW, 1, 77, dev)
lo, hi = shard_bounds(G, world, rank)

m = UNetModel((HW, HW, 3), 1, dropout_rate=DROP, device=dev, seed=SEED)
m.compile(AdamW(LR, WD), "dice_loss")
m.enable_data_parallel(bucket_bytes=1 << 20, sync_bn=SYNC)
m.train_step(x_all[lo:hi], y_all[lo:hi], global_size=G)
torch.cuda.synchronize()
g_dp = m.engine.grads.detach().double() / world  # the all-reduced SUM; AdamW applies 1/world
s_dp = m.engine.stats.detach().clone()
p_dp = m.engine.params.detach().clone()

ref = UNetModel((HW, HW, 3), 1, dropout_rate=DROP, device=dev, seed=SEED)
ref.compile(AdamW(LR, WD), "dice_loss")
if DROP:  # the same DP step through the unfused BN-backward statistics route
    ref.engine.fuse_bn_stats = False
    ref.enable_data_parallel(bucket_bytes=1 << 20, sync_bn=SYNC)
    ref.train_step(x_all[lo:hi], y_all[lo:hi], global_size=G)
    torch.cuda.synchronize()
    g_ref = ref.engine.grads.detach().double() / world
else:
    ref.train_step(x_all, y_all)
    torch.cuda.synchronize()
    g_ref = ref.engine.grads.detach().double()
s_ref = ref.engine.stats.detach().double()

worst_g, worst_name = 0.0, ""
for s in m.engine.specs:
    if not s.trainable:
        continue
    o = m.engine.train_layout.offsets[s.name]
    a, b = g_dp[o:o + s.size], g_ref[o:o + s.size]
    e = float((a - b).norm() / (b.norm() + 1e-30))
    if e > worst_g:
        worst_g, worst_name = e, s.name
s_err = float((s_dp.double() - s_ref).abs().max() / (s_ref.abs().max() + 1e-30))
ok_vals = worst_g <= (1e-4 if DROP else 2e-5) and s_err <= 1e-6

mine = [(g_dp * world).float().cpu(), p_dp.cpu(), s_dp.cpu()]
gs, ps, ss = ([torch.empty_like(t) for _ in range(world)] for t in mine)
for lst, t in zip((gs, ps, ss), mine):
    dist.all_gather(lst, t)
ok_same = all(torch.equal(gs[0], t) for t in gs) and all(torch.equal(ps[0], t) for t in ps) and \
    all(torch.equal(ss[0], t) for t in ss)
print(f"dp_syncbn_check rank {rank}/{world} sync_bn={SYNC} drop={DROP} shard [{lo},{hi}) of {G}: grad rel-L2 vs the "
      f"{'unfused-statistics DP' if DROP else 'full-batch'} step {worst_g:.2e} (worst {worst_name}), moving stats {s_err:.2e}; equal to full batch: {ok_vals}",
      flush=True)
if rank == 0:
    print(f"dp_syncbn_check world={world}: grads/params/stats identical across ranks: {ok_same}", flush=True)
dist.barrier()
dist.destroy_process_group()
sys.exit(0 if not SYNC or (ok_same and ok_vals) else 1)  # (the local-BN variant is for contrast only)
