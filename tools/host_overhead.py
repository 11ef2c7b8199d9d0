"""Host-side cost of one train step: time to enqueue (no sync) vs GPU time per step."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "unet-image-segmentation_amd"), ROOT]
import torch
from bench import synthetic_batch
from unet_amd.model import UNetModel
from unet_amd.optim import AdamW
m = UNetModel((256, 256, 3), 1)
m.compile(AdamW(2e-3, 1e-4), "dice_loss")
x, y = synthetic_batch(16, 256, 256, 1, 1, "cuda")
for _ in range(3):
    m.train_step(x, y)
torch.cuda.synchronize()
for overlap in (True, False):
    m.engine.overlap = overlap
    enq = []
    t0 = time.perf_counter()
    for _ in range(10):
        a = time.perf_counter()
        m.train_step(x, y)
        enq.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    tot = (time.perf_counter() - t0) / 10
    print(f"overlap={overlap}: enqueue {sum(enq)/len(enq)*1e3:.2f} ms/step (min {min(enq)*1e3:.2f}), wall {tot*1e3:.2f} ms/step")
