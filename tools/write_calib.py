"""Calibration of rocprofv3's WRITE_SIZE for 4-byte stores (MI355X_MICROARCH.md: "other access
widths are uncalibrated"): known byte counts written by simple kernels in the patterns the
tracer's pixel stores take.  Run under rocprofv3 --pmc WRITE_SIZE; tools/write_calib_summary.py
reads the counters back.  Each pattern writes the same 32 MiB image of int32 pixels:
  fill        torch fill_: wide coalesced stores
  scatter     out[perm] = v with a random permutation: 4 B per lane, every lane another line
  block8x8    the image dealt in 8x8 blocks (one block per 64 consecutive lanes, the tracer's
              block-major queue order), written in one pass
  block_rows  the same order, the 8 pixels of each block row written by 8 separate passes
              (one pixel of every row segment per pass: a 32-B sector completed over 8 passes)
"""
import torch

W = H = 2896  # ~32 MiB of int32
N = W * H
dev = "cuda"
out = torch.zeros(N, dtype=torch.int32, device=dev)
vals = torch.arange(N, dtype=torch.int32, device=dev)
perm = torch.randperm(N, device=dev)
# block-major order: position q -> block q >> 6, pixel q & 63 (row-major inside the 8x8 block)
bw = W // 8
q = torch.arange((W // 8) * (H // 8) * 64, device=dev)
blk, pq = q >> 6, q & 63
by, bx = blk // bw, blk % bw
order = ((by * 8 + (pq >> 3)) * W + bx * 8 + (pq & 7)).to(torch.int64)
torch.cuda.synchronize()
for _ in range(3):
    out.fill_(7)
    out[perm] = vals
    out[order] = vals[: order.numel()]
    for k in range(8):  # pass k writes pixel k of every 8-pixel row segment
        sel = order[(pq & 7) == k]
        out[sel] = vals[: sel.numel()]
    torch.cuda.synchronize()
print("bytes per pattern", N * 4, "block pattern bytes", order.numel() * 4)
