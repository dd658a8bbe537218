"""Benchmark: Mray-steps/s (+ frames/s) of the neural-SDF sphere tracer at 1024^2 on plane_1.h5.

BASELINE.json metric "Mray-steps/s + frames/s at 1024^2, plane_1.h5, 1/2/4/8 MI355X";
workload = configs[1]: plane_1.h5, 1024x1024, 128 march steps, fp32, Chrome.png matcap,
default camera (rx = ry = 0, zoom 2, frame 0), v1 scene (sceneSDF -> manySphere,
volumeRender_kernel.cu:222).  One "step" = one frame of that workload rendered to
device memory (and, for N > 1, gathered to rank 0 and assembled).

    python bench.py [--gpus N --steps K --warmup W]
The K frames of the timed region go through nr_render_batch: the persistent tracer's
pixel queue runs through the frames in order (up to 32 per launch), so one frame's
longest rays march while the next frame's pixels keep the matrix cores busy -- every
frame is rendered in full, none is reused.  config.single_frame repeats the timing with
one nr_render call per frame (each launch waits for the previous frame's last ray).

N > 1 runs under torch.distributed.run, one rank per GPU: rows are dealt round-robin one
row at a time (band 1, nr_render_batch's shard arguments: the slowest of 8 ranks is within
1% of the mean, against 6% for 8-row bands -- tools/shard_balance.py), each rank renders its rows of every
frame, then one RCCL gather (torch.distributed.gather over the "nccl" backend) brings
the batch's shards to rank 0 -- one collective for the K frames, single-frame timing:
one per frame -- which re-interleaves each frame (nr_assemble_shards).  The frame size
is fixed as N grows: scaling "strong".

Prints ONE JSON line on rank 0 (driver contract) with `roofline` (dominant kernel
k_trace, f32 MFMA bound, per-launch HIP events on the stream it runs on) and
`cpu_baseline` (the C oracle on the host cores, N = 1 only).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

FLOP_PER_EVAL = 2 * (3 * 32 + 7 * 32 * 32 + 32 * 1)   # 14,592
PEAK = {"fp32": 157.3, "bf16": 2516.6, "fp16": 2516.6}  # TFLOP/s dense, MI355X_MICROARCH.md
MAX_STEPS = 128
BAND = 1  # rows per band dealt round-robin to the ranks (profiles/r1_shard_balance.txt)
MAX_BATCH = 32  # frames per k_trace launch (NR_MAX_BATCH)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16", "fp16"])
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--max-steps", type=int, default=MAX_STEPS)
    ap.add_argument("--geometry", default="plane_1")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-single-frame", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    return ap.parse_args()


def cpu_baseline(size, max_steps, threads, geometry, matcap, iv, nm):
    """C oracle (oracle/nr_oracle.c, OpenMP over rays) on the host cores.

    Sample: one full frame of the benchmark workload when it fits the 10-30 s budget,
    else a 512^2 frame of the same camera/steps."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    import cudaneuralrender_amd as nr
    dims, K, B = nr.read_keras_h5(nr.geometry_path(geometry))
    net = oracle.OracleNet(K, B)
    # calibrate on a 256^2 frame, then pick the sample
    t0 = time.perf_counter()
    _, st = net.render(256, 256, iv, nm, color_type=1, matcap=matcap, max_steps=max_steps, nthreads=threads)
    rate = st["ray_steps"] / (time.perf_counter() - t0)
    est_full = 15e6 * (size / 1024) ** 2 / max(rate, 1.0)
    s = size if est_full <= 30.0 else 512
    t0 = time.perf_counter()
    _, st = net.render(s, s, iv, nm, color_type=1, matcap=matcap, max_steps=max_steps, nthreads=threads)
    dt = time.perf_counter() - t0
    return {"value": round(st["ray_steps"] / dt / 1e6, 4), "unit": "Mray-steps/s", "cores": threads,
            "kind": "port",
            "sample": f"{geometry} {s}x{s}, {max_steps} steps, Chrome matcap, default camera: "
                      f"{st['ray_steps']} ray-steps in {dt:.2f} s (C oracle, OpenMP, {threads} threads, "
                      f"host {os.cpu_count()} logical CPUs)"}


def main():
    a = parse()
    import torch
    import torch.distributed as dist
    import cudaneuralrender_amd as nr

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    size = a.size
    matcap = nr.load_png(nr.matcap_path("Chrome"))
    iv, nm = nr.camera(0.0, 0.0, 2.0)
    rows = nr.shard_rows(size, BAND, world, rank)
    max_rows = max(nr.shard_rows(size, BAND, world, s) for s in range(world))

    stream = torch.cuda.Stream()
    r = nr.Renderer(local)
    r.load_h5(nr.geometry_path(a.geometry)).set_precision(a.precision)
    r.set_view(iv, nm, 0).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(matcap)
    r.set_stream(stream.cuda_stream)

    nbuf = max(a.steps, a.warmup, 1)
    shard_px = max_rows * size
    shards = torch.zeros(nbuf, shard_px, dtype=torch.int32, device="cuda")
    frames = shards if world == 1 else (
        torch.zeros(nbuf, size * size, dtype=torch.int32, device="cuda") if rank == 0 else None)
    gather = torch.zeros(world, nbuf * shard_px, dtype=torch.int32, device="cuda") if (rank == 0 and world > 1) else None

    def collect(i0, n):
        """Frames i0..i0+n-1 to rank 0: ONE RCCL gather of the n shards of every rank, then
        the re-interleave kernel per frame (rank s's shard of frame i at gather[s][i])."""
        if world == 1:
            return
        src = shards[i0:i0 + n].reshape(-1)
        dist.gather(src, [g[: n * shard_px] for g in gather.unbind(0)] if rank == 0 else None, dst=0)
        if rank == 0:
            for i in range(n):
                r.assemble_device(gather.data_ptr() + i * shard_px * 4, nbuf * shard_px, frames[i0 + i].data_ptr(),
                                  size, size, BAND, world)

    def run_batched(n):
        if n == 0:
            return
        with torch.cuda.stream(stream):
            r.render_batch_device([shards[i].data_ptr() for i in range(n)], size, size, [(iv, nm, 0)] * n,
                                  a.max_steps, BAND, world, rank)
            collect(0, n)

    def run_single(n):
        with torch.cuda.stream(stream):
            for i in range(n):
                r.render_shard_device(shards[i].data_ptr(), size, size, BAND, world, rank, a.max_steps)
                collect(i, 1)

    # work per frame (deterministic): ray-steps of this rank's shard, summed over ranks
    st = r.render_shard(size, size, BAND, world, rank, a.max_steps)[1]
    steps_t = torch.tensor([st["ray_steps"], st["shade_evals"]], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(steps_t)
    ray_steps, shade_evals = (float(v) for v in steps_t.tolist())

    def timed(fn, profile):
        fn(a.warmup)
        torch.cuda.synchronize()
        r.prof_collect()          # drop anything recorded so far
        r.set_profiling(profile)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(a.steps)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        r.set_profiling(False)
        prof = r.prof_collect()
        dt_t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        if world > 1:
            dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
        return float(dt_t.item()), prof

    dt, prof = timed(run_batched, True)
    last = frames[a.steps - 1] if frames is not None else None

    # parity spot-check of the last timed frame (outside the timed region)
    parity = None
    if rank == 0:
        ref = r.render(size, size, a.max_steps, with_stats=False)
        torch.cuda.synchronize()
        got = last.cpu().numpy().view(np.uint32)[: size * size].reshape(size, size)
        parity = bool(np.array_equal(ref, got))

    dt_single = None
    if not a.no_single_frame:
        dt_single, _ = timed(run_single, False)

    # roofline of the dominant kernel (k_trace) from this rank's per-launch events
    launches = max(prof["march_launches"], 1)
    march_avg_ms = prof["march_ms"] / launches
    # k_trace evaluates the MLP for every march step AND the 4 tetrahedral samples of
    # every coloured ray (in-kernel shading), 14,592 algorithmic FLOP each
    local_evals = (st["ray_steps"] + st["shade_evals"]) * prof["renders"]
    flop_per_launch = local_evals * FLOP_PER_EVAL / launches
    achieved = flop_per_launch / (march_avg_ms * 1e-3) / 1e12 if march_avg_ms > 0 else 0.0
    peak = PEAK[a.precision]

    # HBM traffic of k_trace from the PMC pass committed under profiles/ (rocprofv3 --pmc
    # FETCH_SIZE / WRITE_SIZE, separate passes, gfx950 2x fetch correction) when it was
    # collected on this workload; bench.py cannot read PMC counters itself
    traffic = None
    try:
        tp = json.load(open(os.path.join(REPO, "profiles", "r1_pmc_traffic.json")))
        if (a.precision == "fp32" and size == 1024 and a.max_steps == 128 and world == 1
                and tp.get("frames_per_launch") == min(a.steps, MAX_BATCH)):
            traffic = tp["hbm_bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        traffic = None

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    value = ray_steps * a.steps / dt / 1e6
    out = {
        "metric": "Mray-steps/s at 1024^2, plane_1.h5 (frames/s in config.fps)",
        "value": round(value, 3),
        "unit": "Mray-steps/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(dt / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32" if a.precision == "fp32" else a.precision,
        "data": "synthetic camera (default pose), real bundled weights plane_1.h5 + Chrome.png",
        "config": {
            "workload": f"{a.geometry} {size}x{size}, {a.max_steps} march steps, {a.precision}, Chrome.png, "
                        "v1 scene, default camera (BASELINE configs[1])",
            "fps": round(a.steps / dt, 3),
            "ray_steps_per_frame": int(ray_steps),
            "shade_evals_per_frame": int(shade_evals),
            "frames_per_launch": min(a.steps, MAX_BATCH),
            "schedule": "nr_render_batch: the K timed frames through one frame-major pixel queue "
                        "(every frame rendered in full)",
            "parallelism": f"row-band shards x{world} + one RCCL gather per batch of frames" if world > 1
                           else "single GPU",
            "parity_vs_single_gpu_render": parity,
            "single_frame": None if dt_single is None else {
                "value": round(ray_steps * a.steps / dt_single / 1e6, 3),
                "ms_per_step": round(dt_single / a.steps * 1e3, 4),
                "fps": round(a.steps / dt_single, 3),
                "schedule": "one nr_render_shard launch per frame",
            },
        },
        "roofline": {
            "bound": "mfma",
            "kernel": "k_trace (batched instance)",
            "achieved": round(achieved, 3),
            "peak": peak,
            "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4),
            "traffic": traffic,
            "traffic_unit": "bytes per launch (profiles/r1_pmc_traffic.json)",
            "flop_per_launch": round(flop_per_launch, 1),
            "avg_launch_ms": round(march_avg_ms, 5),
            "launches": int(prof["march_launches"]),
            "flop_basis": "(ray-steps + shade evals) x 14,592 FLOP per frame x frames per launch / mean k_trace "
                          "launch duration (per-launch HIP events on the context stream)",
        },
        "cpu_baseline": None,
    }
    if world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(size, a.max_steps, a.cpu_threads, a.geometry, matcap, iv, nm)
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
