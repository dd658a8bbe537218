"""Benchmark: Mray-steps/s (+ frames/s) of the neural-SDF sphere tracer at 1024^2 on plane_1.h5.

BASELINE.json metric "Mray-steps/s + frames/s at 1024^2, plane_1.h5, 1/2/4/8 MI355X";
workload = configs[1]: plane_1.h5, 1024x1024, 128 march steps, fp32, Chrome.png matcap,
default camera (rx = ry = 0, zoom 2, frame 0), v1 scene (sceneSDF -> manySphere,
volumeRender_kernel.cu:222).  One "step" = one frame of that workload rendered to
device memory (and, for N > 1, gathered to rank 0 and assembled).

    python bench.py [--gpus N --steps K --warmup W]
The K frames of the timed region go through nr_render_batch: the persistent tracer's
pixel queue deals 64-pixel chunks to the frames in turn (up to 32 frames per launch), so
one frame's longest rays march while other frames' pixels keep the matrix cores busy --
every frame is rendered in full, none is reused.  config.single_frame repeats the timing with
one nr_render call per frame (each launch waits for the previous frame's last ray).

N > 1 runs one rank per GPU under torch.distributed.run: the driver's launcher, or, when
`python bench.py --gpus N` is started without one (WORLD_SIZE unset), bench.py starts
`python -m torch.distributed.run --nproc-per-node N ... bench.py` itself as a child process
before anything touches a GPU and exits with its status.  Rows are dealt round-robin one
row at a time (band 1, nr_render_batch's shard arguments: the slowest of 8 ranks is within
1% of the mean, against 6% for 8-row bands -- tools/shard_balance.py), each rank renders its rows of every
frame, then one RCCL gather (torch.distributed.gather over the "nccl" backend) brings
the batch's shards to rank 0 -- one collective for the K frames, single-frame timing:
one per frame -- which re-interleaves each frame (nr_assemble_shards).  The frame size
is fixed as N grows: scaling "strong".

`value` = the ray-steps the timed launches themselves counted (nr_render_batch's stats,
summed over ranks) / the max-over-ranks wall time of the timed region.  Every timed frame
is checked against a reference render afterwards (config.parity_frames_checked).
config.random_poses repeats the timing over 8 poses from default_rng(1) (rx in [-30, 30],
ry in [0, 360), zoom 2), the K frames cycling through them.

--config c3 / c4 / c5 time the other BASELINE configs with the same harness (c3 car_1 2048^2
bf16 256 steps; c4 plane_2 4096^2 bf16, row-band shards + gather; c5 one geometry per rank,
GEOMS[rank % 5], 2048^2 fp16, independent replicas with no collective: scaling "weak",
config.per_rank_value).  With fp32, config.fp32x3 times the same K frames in
NR_PRECISION_FP32X3 (the fp32-class split on the fp16 matrix core; its pixel contract is
tests/test_gpu_fp32x3.py) and reports its agreement with the fp32 frame.

Prints ONE JSON line on rank 0 (driver contract) with `roofline` (dominant kernel
k_trace, f32 MFMA bound, per-launch HIP events on the stream it runs on; per rank for
N > 1) and `cpu_baseline` (the C oracle on the host cores, N = 1 only: all-core value
plus a single-thread figure and the CPU model).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

FLOP_PER_EVAL = 2 * (3 * 32 + 7 * 32 * 32 + 32 * 1)   # 14,592
# TFLOP/s dense, MI355X_MICROARCH.md; fp32x3 runs its hidden layers as three fp16 MFMA terms, so
# its roofline is the fp16 matrix peak (achieved counts the algorithmic 14,592 FLOP per eval)
PEAK = {"fp32": 157.3, "bf16": 2516.6, "fp16": 2516.6, "fp32x3": 2516.6}
GEOMS = ["plane_1", "plane_2", "plane_3", "car_1", "3a3d4a90a2db90b4203936772104a82d.obj"]
# BASELINE.json configs: c2 is the headline (configs[1]); c3 / c4 / c5 are configs[2..4].
# c5 renders one geometry per rank (GEOMS[rank % 5]) as independent replicas: no collective.
PRESETS = {
    "c2": dict(geometry="plane_1", size=1024, precision="fp32", max_steps=128),
    "c3": dict(geometry="car_1", size=2048, precision="bf16", max_steps=256),
    "c4": dict(geometry="plane_2", size=4096, precision="bf16", max_steps=128),
    "c5": dict(geometry=None, size=2048, precision="fp16", max_steps=128),
}
MAX_STEPS = 128
BAND = 1  # rows per band dealt round-robin to the ranks (profiles/r1_shard_balance.txt)
MAX_BATCH = 32  # frames per k_trace launch (NR_MAX_BATCH)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--config", default="c2", choices=sorted(PRESETS),
                    help="BASELINE config preset (c2 = the headline); the flags below override it")
    ap.add_argument("--precision", default=None, choices=["fp32", "bf16", "fp16", "fp32x3"])
    ap.add_argument("--size", type=int, default=None)
    ap.add_argument("--max-steps", type=int, default=None)
    ap.add_argument("--geometry", default=None)
    ap.add_argument("--no-fp32x3", action="store_true",
                    help="skip config.fp32x3 (the same frames timed in NR_PRECISION_FP32X3)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-live-traffic", action="store_true",
                    help="take roofline.traffic from the committed PMC figure instead of two rocprofv3 --pmc "
                         "child passes in this run")
    ap.add_argument("--no-single-frame", action="store_true")
    ap.add_argument("--no-spin", action="store_true",
                    help="skip config.spin (the reference's --spin sequence, one launch per frame)")
    ap.add_argument("--no-random-poses", action="store_true",
                    help="skip config.random_poses (profiling passes that average the default-pose launches)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--group", action="store_true",
                    help="one process drives all N GPUs through the C ABI's nr_group (RCCL gather, "
                         "NR_GROUP_ASYNC) instead of one torch.distributed rank per GPU")
    ap.add_argument("--no-group", action="store_true",
                    help="N > 1 under torch.distributed: skip config.group (rank 0's nr_group child run)")
    a = ap.parse_args()
    for k, v in PRESETS[a.config].items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    a.replicas = a.config == "c5"
    return a


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(size, max_steps, threads, geometry, matcap, iv, nm):
    """C oracle (oracle/nr_oracle.c, OpenMP over rays) on the host cores, all-core and
    single-thread.

    All-core sample: one full frame of the benchmark workload when it fits ~30 s, else a
    512^2 frame of the same camera/steps; single-thread sample: a 256^2 frame of the same
    camera/steps (about 0.98 M ray-steps, a few seconds)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    import cudaneuralrender_amd as nr
    dims, K, B = nr.read_keras_h5(nr.geometry_path(geometry))
    net = oracle.OracleNet(K, B)
    # single thread on 256^2 (also the calibration for the all-core sample)
    t0 = time.perf_counter()
    _, st1 = net.render(256, 256, iv, nm, color_type=1, matcap=matcap, max_steps=max_steps, nthreads=1)
    dt1 = time.perf_counter() - t0
    rate1 = st1["ray_steps"] / dt1
    est_full = 15e6 * (size / 1024) ** 2 / max(rate1 * threads * 0.7, 1.0)
    s = size if est_full <= 30.0 else 512
    t0 = time.perf_counter()
    _, st = net.render(s, s, iv, nm, color_type=1, matcap=matcap, max_steps=max_steps, nthreads=threads)
    dt = time.perf_counter() - t0
    return {"value": round(st["ray_steps"] / dt / 1e6, 4), "unit": "Mray-steps/s", "cores": threads,
            "kind": "port",
            "sample": f"{geometry} {s}x{s}, {max_steps} steps, Chrome matcap, default camera: "
                      f"{st['ray_steps']} ray-steps in {dt:.2f} s (C oracle, OpenMP, {threads} threads)",
            "single_thread": {"value": round(rate1 / 1e6, 4), "unit": "Mray-steps/s", "cores": 1,
                              "sample": f"{geometry} 256x256, {max_steps} steps: {st1['ray_steps']} ray-steps "
                                        f"in {dt1:.2f} s"},
            "cpu_model": cpu_model(),
            "host_logical_cpus": os.cpu_count(),
            "threads_note": "the GPU box's CPU share is 16 threads (OMP_NUM_THREADS); os.cpu_count() "
                            "reports the whole machine"}


def live_traffic(frames, precision, size, max_steps):
    """k_trace's HBM bytes per launch measured in this run: two rocprofv3 --pmc passes (FETCH_SIZE,
    then WRITE_SIZE -- separate runs, MI355X_MICROARCH.md's HBM/rocprofv3 recipe) over
    tools/render_frames.py rendering 3 launches of the bench's batch (`frames` frames of the same
    workload per nr_render_batch), each pass a child process under a hard time limit.  gfx950
    corrections: FETCH_SIZE is KiB and under-counts wide reads 2x, WRITE_SIZE is KiB.  Returns
    (bytes per launch, detail) or None when rocprofv3 is absent or a pass fails (the caller then
    falls back to the committed figure)."""
    import csv
    import glob
    import shutil
    import tempfile
    prof = shutil.which("rocprofv3")
    if prof is None or "ROCPROF_OUTPUT_PATH" in os.environ:   # absent, or this run is itself profiled
        return None
    kname = "k_trace<0, false, false, true, false, false"  # (a prefix: later template arguments follow)
    tmp = tempfile.mkdtemp(prefix="nr_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    vals = {}
    t0 = time.perf_counter()
    try:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            cmd = ["timeout", "-k", "5", "-s", "KILL", "90", prof, "--pmc", counter, "--output-format", "csv",
                   "-d", os.path.join(tmp, counter), "-o", "run", "--", sys.executable,
                   os.path.join(REPO, "tools", "render_frames.py"), "--frames", "3", "--batch", str(frames),
                   "--precision", precision, "--size", str(size), "--steps", str(max_steps)]
            with open(os.path.join(tmp, counter + ".log"), "w") as log:
                rc = subprocess.run(cmd, cwd="/tmp", env=env, stdout=log, stderr=subprocess.STDOUT,
                                    timeout=120).returncode
            got = []
            for f in glob.glob(os.path.join(tmp, counter, "**", "*counter_collection.csv"), recursive=True):
                with open(f) as fh:
                    got += [float(r["Counter_Value"]) for r in csv.DictReader(fh)
                            if kname in r["Kernel_Name"] and r["Counter_Name"] == counter]
            if rc != 0 or not got:
                print(f"bench: live PMC pass {counter} failed (exit {rc}, {len(got)} dispatches); "
                      "using the committed traffic figure", file=sys.stderr)
                return None
            vals[counter] = (sum(got) / len(got), len(got))
    except (OSError, subprocess.SubprocessError) as e:
        print(f"bench: live PMC passes unavailable ({e}); using the committed traffic figure", file=sys.stderr)
        return None
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    fetch, write = vals["FETCH_SIZE"][0], vals["WRITE_SIZE"][0]
    hbm = fetch * 1024 * 2 + write * 1024
    return int(hbm), {"fetch_size_kb": round(fetch, 2), "write_size_kb": round(write, 2),
                      "dispatches": [vals["FETCH_SIZE"][1], vals["WRITE_SIZE"][1]],
                      "frames_per_launch": frames, "seconds": round(time.perf_counter() - t0, 1),
                      "algorithmic_bytes_per_launch": size * size * 4 * frames + 30 * 1024 + 1024 * 1024}


def random_poses(n=8):
    """8 poses from default_rng(1), rx in U[-30, 30], ry in U[0, 360), zoom 2."""
    rng = np.random.default_rng(1)
    return [(float(rng.uniform(-30, 30)), float(rng.uniform(0, 360))) for _ in range(n)]


class RankFailed(RuntimeError):
    """Another rank's render of this batch raised."""


_STATUS_GROUP = []


def status_group(dist):
    """A gloo (CPU) process group for the status exchange, created once: a rank whose GPU faulted
    can still take part in it, where an all-reduce on the RCCL group would need that GPU."""
    if not _STATUS_GROUP:
        _STATUS_GROUP.append(dist.new_group(backend="gloo"))
    return _STATUS_GROUP[0]


def checked_step(dist, world, device, fn):
    """Runs fn() -- this rank's render of a batch -- and then, before the batch's gather, lets
    every rank learn whether any rank's fn raised: one all-reduce (MAX) of a status int over a
    gloo group on the CPU (no device sync; the render itself already waited for its counters).
    The failing rank re-raises its own error and the others raise RankFailed, so every rank exits
    within seconds instead of blocking in the gather until the collective times out (SURVEY.md
    section 5: a per-rank status all-reduce before the gather).  One exchange per batch of up to
    32 frames: ~0.1 ms of gloo over loopback against ~36 ms per 20-frame batch."""
    err = None
    try:
        fn()
    except Exception as e:  # noqa: BLE001 -- re-raised below, after the status exchange
        err = e
    failed = 1 if err is not None else 0
    if world > 1:
        import torch
        t = torch.tensor([failed], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=status_group(dist) if device != "cpu" else None)
        failed = int(t.item())
    if err is not None:
        raise err
    if failed:
        raise RankFailed("another rank failed to render its shard of this batch")


def self_launch(a):
    """--gpus N > 1 without a launcher: run this script under torch.distributed.run, one
    rank per GPU, as a child process (nothing here has touched a GPU), and return its status."""
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def main_group(a):
    """--group: one process, N contexts (GPUs 0..N-1) joined by nr_group (csrc/nr_group.hip, the
    C-ABI multi-GPU product path: row-band shards rendered in parallel, one RCCL gather per call,
    the re-interleave on GPU 0), NR_GROUP_ASYNC with up to 32 frames per call, so call k + 1
    renders while call k's shards travel.  Same JSON contract as the rank path."""
    import torch
    import cudaneuralrender_amd as nr
    n = a.gpus
    if torch.cuda.device_count() < n:
        raise SystemExit(f"--group --gpus {n}: only {torch.cuda.device_count()} GPUs visible")
    size = a.size
    matcap = nr.load_png(nr.matcap_path("Chrome"))
    iv, nm = nr.camera(0.0, 0.0, 2.0)
    geometry = a.geometry or GEOMS[0]
    rs = []
    for d in range(n):
        r = nr.Renderer(d)
        r.load_h5(nr.geometry_path(geometry)).set_precision(a.precision)
        r.set_view(iv, nm, 0).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(matcap)
        rs.append(r)
    g = nr.Group(rs, asynchronous=True)
    nbuf = max(a.steps, a.warmup, 1)
    frames = torch.zeros(nbuf, size * size, dtype=torch.int32, device="cuda:0")
    cams = [(iv, nm, 0)]
    counted = {"ray_steps": 0, "shade_evals": 0}

    def run(k):
        for i0 in range(0, k, MAX_BATCH):
            m = min(MAX_BATCH, k - i0)
            st = g.render_batch_device([frames[i0 + i].data_ptr() for i in range(m)], size, size, cams * m,
                                       a.max_steps, band=BAND, with_stats=True)
            counted["ray_steps"] += st["ray_steps"]
            counted["shade_evals"] += st["shade_evals"]

    def sync_all():
        g.synchronize()
        for d in range(n):
            torch.cuda.synchronize(d)

    run(a.warmup)
    sync_all()
    rs[0].prof_collect()
    rs[0].set_profiling(True)
    counted["ray_steps"] = counted["shade_evals"] = 0
    t0 = time.perf_counter()
    run(a.steps)
    sync_all()
    dt = time.perf_counter() - t0
    rs[0].set_profiling(False)
    prof = rs[0].prof_collect()
    ref = torch.from_numpy(rs[0].render(size, size, a.max_steps, with_stats=False).view(np.int32).reshape(-1)).to("cuda:0")
    parity = all(bool(torch.equal(frames[i], ref)) for i in range(a.steps))
    launches = max(prof["march_launches"], 1)
    march_avg_ms = prof["march_ms"] / launches
    # rank 0's k_trace launches render shard 0: its share of the counted work (1 / n of the rows)
    achieved = (counted["ray_steps"] + counted["shade_evals"]) / n * FLOP_PER_EVAL / launches / (march_avg_ms * 1e-3) / 1e12 \
        if march_avg_ms > 0 else 0.0
    peak = PEAK[a.precision]
    out = {
        "metric": "Mray-steps/s at 1024^2, plane_1.h5 (frames/s in config.fps)",
        "value": round(counted["ray_steps"] / dt / 1e6, 3), "unit": "Mray-steps/s", "n_gpus": n, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32" if a.precision == "fp32" else a.precision,
        "data": f"synthetic camera (default pose), real bundled weights {geometry}.h5 + Chrome.png",
        "config": {
            "workload": f"{geometry} {size}x{size}, {a.max_steps} march steps, {a.precision}, Chrome.png, v1 scene, "
                        f"default camera (BASELINE configs[1])",
            "config": a.config, "fps": round(a.steps / dt, 3), "ray_steps_counted": int(counted["ray_steps"]),
            "parallelism": f"nr_group (one process, C ABI): row-band shards x{n} (band {BAND}), one RCCL gather "
                           f"per call of <= {MAX_BATCH} frames, NR_GROUP_ASYNC (call k+1 renders while call k's "
                           f"shards travel), re-interleave on GPU 0",
            "parity_vs_single_gpu_render": parity, "parity_frames_checked": a.steps,
        },
        "roofline": {"bound": "mfma", "kernel": "k_trace (batched instance, GPU 0's shard)",
                     "achieved": round(achieved, 3), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(achieved / peak, 4), "traffic": None, "avg_launch_ms": round(march_avg_ms, 5)},
        "cpu_baseline": None,
    }
    if n == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(size, a.max_steps, a.cpu_threads, geometry, matcap, iv, nm)
    g.close()
    for r in rs:
        r.close()
    return out


def group_child(a):
    """Rank 0 of an N > 1 rank run: the same workload through nr_group in a child process over all
    N GPUs (WORLD_SIZE etc. dropped from its environment), its JSON line attached as config.group,
    bounded by a time limit: the C-ABI multi-GPU path measured on the node the driver runs."""
    cmd = [sys.executable, os.path.abspath(__file__), "--group", "--gpus", str(a.gpus), "--steps", str(a.steps),
           "--warmup", str(a.warmup), "--config", a.config, "--precision", a.precision, "--size", str(a.size),
           "--max-steps", str(a.max_steps), "--no-cpu-baseline"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    try:
        p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    except subprocess.TimeoutExpired:
        return {"error": "timed out after 240 s"}
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        return {"error": f"exit {p.returncode}", "stderr_tail": p.stderr[-600:]}
    d = json.loads(lines[-1])
    return {k: d[k] for k in ("value", "ms_per_step", "n_gpus")} | {
        "fps": d["config"]["fps"], "parity_vs_single_gpu_render": d["config"]["parity_vs_single_gpu_render"],
        "parallelism": d["config"]["parallelism"], "roofline_frac_gpu0": d["roofline"]["frac"]}


def json_stdout():
    """The bench's stdout carries its one JSON line only: native libraries that write to fd 1
    (RCCL's version banner at communicator set-up, ...) are pointed at stderr, and the JSON line
    goes to a private copy of the real stdout.  Called in the process that prints the line (not
    in a launcher whose children inherit fd 1)."""
    sys.stdout.flush()
    real = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(real, "w", buffering=1)


def main():
    a = parse()
    if a.group:
        if "WORLD_SIZE" in os.environ:
            raise SystemExit("--group runs in one process: start it without torch.distributed.run")
        out = json_stdout()
        print(json.dumps(main_group(a)), file=out, flush=True)
        return
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(self_launch(a))
    jout = json_stdout()
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
    # replicas (c5): every rank renders whole frames of its own geometry, no shards, no collective
    nsh, sh = (1, 0) if a.replicas else (world, rank)
    geometry = a.geometry or GEOMS[rank % len(GEOMS)]
    max_rows = max(nr.shard_rows(size, BAND, nsh, s) for s in range(nsh))

    stream = torch.cuda.Stream()
    r = nr.Renderer(local)
    r.load_h5(nr.geometry_path(geometry)).set_precision(a.precision)
    r.set_view(iv, nm, 0).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(matcap)
    r.set_stream(stream.cuda_stream)

    nbuf = max(a.steps, a.warmup, 1)
    shard_px = max_rows * size
    shards = torch.zeros(nbuf, shard_px, dtype=torch.int32, device="cuda")
    frames = shards if (world == 1 or a.replicas) else (
        torch.zeros(nbuf, size * size, dtype=torch.int32, device="cuda") if rank == 0 else None)
    gather = (torch.zeros(world, nbuf * shard_px, dtype=torch.int32, device="cuda")
              if (rank == 0 and world > 1 and not a.replicas) else None)

    def collect(i0, n):
        """Frames i0..i0+n-1 to rank 0: ONE RCCL gather of the n shards of every rank, then
        the re-interleave kernel per frame (rank s's shard of frame i at gather[s][i])."""
        if world == 1 or a.replicas:
            return
        src = shards[i0:i0 + n].reshape(-1)
        dist.gather(src, [g[: n * shard_px] for g in gather.unbind(0)] if rank == 0 else None, dst=0)
        if rank == 0:
            if size % (BAND * world) == 0:
                # every frame is a whole number of band rounds: the n frames stacked are one
                # (n*H)-row image whose shard s is rank s's gathered n x rows rows -- one
                # re-interleave launch instead of n (tests/test_dist_cpu.py checks the identity)
                r.assemble_device(gather.data_ptr(), nbuf * shard_px, frames[i0].data_ptr(), size, n * size, BAND,
                                  world)
                return
            for i in range(n):
                r.assemble_device(gather.data_ptr() + i * shard_px * 4, nbuf * shard_px, frames[i0 + i].data_ptr(),
                                  size, size, BAND, world)

    default_cams = [(iv, nm, 0)]
    pose_cams = [(*nr.camera(rx, ry, 2.0), 0) for rx, ry in random_poses()]
    counted = {"ray_steps": 0, "shade_evals": 0}

    def run_batched(n, cams=default_cams):
        """n frames (cycling through cams) in one nr_render_batch call; the call's own
        counters (read back at its end) are what `value` is computed from."""
        if n == 0:
            return
        with torch.cuda.stream(stream):
            def render():
                st = r.render_batch_device([shards[i].data_ptr() for i in range(n)], size, size,
                                           [cams[i % len(cams)] for i in range(n)], a.max_steps, BAND, nsh, sh,
                                           with_stats=True)
                counted["ray_steps"] += st["ray_steps"]
                counted["shade_evals"] += st["shade_evals"]
            checked_step(dist, world, "cuda", render)
            collect(0, n)

    def run_single(n):
        with torch.cuda.stream(stream):
            for i in range(n):
                def render():
                    st = r.render_shard_device(shards[i].data_ptr(), size, size, BAND, nsh, sh, a.max_steps,
                                               with_stats=True)
                    counted["ray_steps"] += st["ray_steps"]
                    counted["shade_evals"] += st["shade_evals"]
                checked_step(dist, world, "cuda", render)
                collect(i, 1)

    def timed(fn, profile):
        """W untimed warmup frames, then exactly K frames between barrier + synchronize;
        returns (max-over-ranks seconds, this rank's k_trace profile, ray-steps and shade
        evals the K frames counted, summed over ranks, and per-rank ray-steps)."""
        fn(a.warmup)
        torch.cuda.synchronize()
        r.prof_collect()          # drop anything recorded so far
        r.set_profiling(profile)
        counted["ray_steps"] = counted["shade_evals"] = 0
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
        mine = torch.tensor([dt, counted["ray_steps"], counted["shade_evals"]], dtype=torch.float64, device="cuda")
        per_rank = [mine.clone() for _ in range(world)]
        if world > 1:
            dist.all_gather(per_rank, mine)
        per_rank = torch.stack(per_rank).cpu().numpy()
        return (float(per_rank[:, 0].max()), prof, float(per_rank[:, 1].sum()), float(per_rank[:, 2].sum()),
                per_rank)

    def check_frames(n, cams):
        """Every timed frame against a full single-GPU nr_render of its camera (rank 0, after
        the timed region): returns (all equal, frames checked)."""
        if rank != 0:
            return None, 0
        refs = {}
        ok = True
        for i in range(n):
            k = i % len(cams)
            if k not in refs:
                r.set_view(cams[k][0], cams[k][1], 0)
                img = r.render(size, size, a.max_steps, with_stats=False)
                refs[k] = torch.from_numpy(img.view(np.int32).reshape(-1)).to("cuda")
            got = frames[i][: size * size]
            ok = ok and bool(torch.equal(got, refs[k]))
        r.set_view(iv, nm, 0)
        torch.cuda.synchronize()
        return ok, n

    dt, prof, ray_steps_k, shade_evals_k, per_rank = timed(run_batched, True)
    rank_steps = per_rank[:, 1]
    parity, nchecked = check_frames(a.steps, default_cams)

    dt_single = None
    if not a.no_single_frame:
        dt_single, _, rs_single, _, _ = timed(run_single, False)

    # The reference's own single-frame use, main.cpp --spin (doABarrelRoll, :470-477): frame i at
    # viewRotation.y = i degrees with frameNumber = i, one launch per frame, timed with and without
    # nr_set_temporal_order (each launch deals its 8x8 blocks longest-first by the PREVIOUS frame's
    # block costs -- a different pose -- so the order is not taken from the frames it times).
    # Single GPU only; the last timed frame is checked against a plain nr_render of its pose.
    spin = None
    if world == 1 and not a.no_spin and not a.no_single_frame:
        spin_i = [0]

        def run_spin(n):
            with torch.cuda.stream(stream):
                for _ in range(n):
                    i = spin_i[0]
                    spin_i[0] += 1
                    ivs, nms = nr.camera(0.0, float(i % 360), 2.0)
                    r.set_view(ivs, nms, i)
                    st = r.render_shard_device(shards[i % nbuf].data_ptr(), size, size, BAND, 1, 0, a.max_steps,
                                               with_stats=True)
                    counted["ray_steps"] += st["ray_steps"]
                    counted["shade_evals"] += st["shade_evals"]

        spin = {"sequence": "frame i at viewRotation.y = i deg, frameNumber = i (main.cpp --spin, :470-477), "
                            "one nr_render_shard launch per frame"}
        for key, order in (("plain", 0), ("temporal_order", 1), ("temporal_order_dilated", 2)):
            spin_i[0] = 0
            r.set_temporal_order(order)
            dts, _, rss, _, _ = timed(run_spin, False)
            spin[key] = {"value": round(rss / dts / 1e6, 3), "ms_per_step": round(dts / a.steps * 1e3, 4),
                         "fps": round(a.steps / dts, 3)}
        r.set_temporal_order(0)
        last = spin_i[0] - 1
        ivs, nms = nr.camera(0.0, float(last % 360), 2.0)
        r.set_view(ivs, nms, last)
        img = r.render(size, size, a.max_steps, with_stats=False)
        ref_last = torch.from_numpy(img.view(np.int32).reshape(-1)).to("cuda")
        spin["parity_last_frame_vs_plain_render"] = bool(torch.equal(shards[last % nbuf][: size * size], ref_last))
        r.set_view(iv, nm, 0)
        torch.cuda.synchronize()

    # the same timing over 8 random poses, frames cycling through them
    dt_pose = None
    if not a.no_random_poses:
        dt_pose, _, rs_pose, se_pose, _ = timed(lambda n: run_batched(n, pose_cams), False)
        pose_parity, pose_checked = check_frames(a.steps, pose_cams)

    # the same K frames in NR_PRECISION_FP32X3 (fp32-class MLP on the fp16 matrix core, not
    # bit-exact: tests/test_gpu_fp32x3.py holds its pixel contract), next to the fp32 headline
    x3 = None
    if a.precision == "fp32" and not a.no_fp32x3:
        ref = None
        if rank == 0:
            img = r.render(size, size, a.max_steps, with_stats=False)
            ref = torch.from_numpy(img.view(np.int32).reshape(-1)).to("cuda")
        r.set_precision("fp32x3")
        dt3, prof3, rs3, se3, pr3 = timed(run_batched, True)
        l3 = max(prof3["march_launches"], 1)
        ms3 = prof3["march_ms"] / l3
        ach3 = float(pr3[rank, 1] + pr3[rank, 2]) * FLOP_PER_EVAL / l3 / (ms3 * 1e-3) / 1e12 if ms3 > 0 else 0.0
        x3 = {"value": round(rs3 / dt3 / 1e6, 3), "ms_per_step": round(dt3 / a.steps * 1e3, 4),
              "fps": round(a.steps / dt3, 3), "ray_steps_per_frame": int(rs3 / a.steps),
              "k_trace_avg_launch_ms": round(ms3, 5),
              "roofline_frac_fp16_peak": round(ach3 / PEAK["fp32x3"], 4),
              "achieved_TFLOPs_algorithmic": round(ach3, 3)}
        if rank == 0:
            x3["identical_pixels_vs_fp32"] = round(float((frames[0][: size * size] == ref).float().mean()), 5)
        r.set_precision(a.precision)

    # roofline of the dominant kernel (k_trace) from this rank's per-launch events
    launches = max(prof["march_launches"], 1)
    march_avg_ms = prof["march_ms"] / launches
    # k_trace evaluates the MLP for every march step AND the 4 tetrahedral samples of
    # every coloured ray (in-kernel shading), 14,592 algorithmic FLOP each; this rank's
    # evals are its own counted ray-steps + shade evals of the timed frames
    local_evals = float(per_rank[rank, 1] + per_rank[rank, 2])
    flop_per_launch = local_evals * FLOP_PER_EVAL / launches
    achieved = flop_per_launch / (march_avg_ms * 1e-3) / 1e12 if march_avg_ms > 0 else 0.0
    peak = PEAK[a.precision]
    roof_t = torch.tensor([achieved, march_avg_ms], dtype=torch.float64, device="cuda")
    roof_all = [roof_t.clone() for _ in range(world)]
    if world > 1:
        dist.all_gather(roof_all, roof_t)
    roof_all = torch.stack(roof_all).cpu().numpy()

    # HBM traffic of k_trace from the PMC pass committed under profiles/ (rocprofv3 --pmc
    # FETCH_SIZE / WRITE_SIZE, separate passes, gfx950 corrections), per frame of this
    # workload, times the frames of one launch; bench.py cannot read PMC counters itself
    traffic, traffic_src, traffic_live = None, None, None
    for name in ("r5_pmc_traffic.json", "r4_pmc_traffic.json", "r3_pmc_traffic.json", "r2_pmc_traffic.json", "r1_pmc_traffic.json"):
        try:
            tp = json.load(open(os.path.join(REPO, "profiles", name)))
        except (OSError, ValueError):
            continue
        if a.config == "c2" and a.precision == "fp32" and size == 1024 and a.max_steps == 128 and world == 1:
            per_frame = tp.get("hbm_bytes_per_frame")
            if per_frame is None and tp.get("frames_per_launch"):
                per_frame = tp["hbm_bytes_per_launch"] / tp["frames_per_launch"]
            if per_frame:
                traffic = int(per_frame * min(a.steps, MAX_BATCH))
                traffic_src = name
        break
    # ... or measured in this run: two rocprofv3 --pmc child passes over the same batched launch
    if (a.config == "c2" and a.precision == "fp32" and world == 1 and not a.no_live_traffic
            and min(a.steps, MAX_BATCH) == a.steps):
        torch.cuda.synchronize()
        live = live_traffic(a.steps, a.precision, size, a.max_steps)
        if live is not None:
            traffic, traffic_live = live

    # the C-ABI multi-GPU path (nr_group) over the same N GPUs, in a child of rank 0, after every
    # timed region; the other ranks wait at the barrier (their contexts stay idle meanwhile)
    group = None
    if world > 1 and not a.replicas and not a.no_group:
        torch.cuda.synchronize()
        if rank == 0:
            group = group_child(a)
        # on the CPU (gloo): an RCCL barrier would leave a spinning collective kernel on every other
        # GPU while the child renders there
        dist.barrier(group=status_group(dist))
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    value = ray_steps_k / dt / 1e6
    out = {
        "metric": "Mray-steps/s at 1024^2, plane_1.h5 (frames/s in config.fps)" if a.config == "c2" else
                  f"Mray-steps/s, BASELINE {a.config} (frames/s in config.fps)",
        "value": round(value, 3),
        "unit": "Mray-steps/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(dt / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak" if a.replicas else "strong",
        "vs_baseline": None,
        "dtype": "f32" if a.precision == "fp32" else a.precision,
        "data": f"synthetic camera (default pose), real bundled weights {geometry}.h5 + Chrome.png"
                if not a.replicas else "synthetic camera (default pose), rank r renders bundled geometry r % 5",
        "config": {
            "workload": (f"{geometry if not a.replicas else 'GEOMS[rank % 5]'} {size}x{size}, {a.max_steps} march "
                         f"steps, {a.precision}, Chrome.png, v1 scene, default camera (BASELINE "
                         f"configs[{ {'c2': 1, 'c3': 2, 'c4': 3, 'c5': 4}[a.config] }])"),
            "config": a.config,
            "fps": round(a.steps / dt, 3),
            "ray_steps_counted": int(ray_steps_k),
            "ray_steps_per_frame": int(ray_steps_k / a.steps),
            "shade_evals_per_frame": int(shade_evals_k / a.steps),
            "frames_per_launch": min(a.steps, MAX_BATCH),
            "schedule": "nr_render_batch: the K timed frames through one pixel queue, 64-pixel chunks "
                        "dealt to the frames in turn (every frame rendered in full)",
            "parallelism": ("replicas: one geometry per rank, no collective" if a.replicas else
                            f"row-band shards x{world} (band {BAND}) + one RCCL gather per batch of frames")
                           if world > 1 else "single GPU",
            "per_rank_value": [round(float(x[1] / x[0] / 1e6), 3) for x in per_rank] if world > 1 else None,
            "geometries": [GEOMS[i % len(GEOMS)] for i in range(world)] if a.replicas else None,
            "fp32x3": x3,
            "group": group,
            "parity_vs_single_gpu_render": parity,
            "parity_frames_checked": nchecked,
            "shard_ray_steps": {"max": int(rank_steps.max()), "mean": round(float(rank_steps.mean()), 1)}
                               if world > 1 else None,
            "single_frame": None if dt_single is None else {
                "value": round(rs_single / dt_single / 1e6, 3),
                "ms_per_step": round(dt_single / a.steps * 1e3, 4),
                "fps": round(a.steps / dt_single, 3),
                "schedule": "one nr_render_shard launch per frame",
            },
            "spin": spin,
            "random_poses": None if dt_pose is None else {
                "value": round(rs_pose / dt_pose / 1e6, 3),
                "ms_per_step": round(dt_pose / a.steps * 1e3, 4),
                "fps": round(a.steps / dt_pose, 3),
                "ray_steps_per_frame": int(rs_pose / a.steps),
                "shade_evals_per_frame": int(se_pose / a.steps),
                "poses": "8 from default_rng(1): rx U[-30,30], ry U[0,360), zoom 2; frames cycle through them",
                "parity_vs_single_gpu_render": pose_parity,
                "parity_frames_checked": pose_checked,
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
            "traffic_unit": ("HBM bytes per launch, measured in this run (rocprofv3 --pmc FETCH_SIZE and "
                             "WRITE_SIZE child passes over the same batched launch; FETCH_SIZE KiB x 2 + "
                             "WRITE_SIZE KiB, gfx950 corrections)" if traffic_live is not None else
                             f"HBM bytes per launch (per-frame PMC figure x frames per launch, profiles/{traffic_src})"
                             if traffic is not None else None),
            "traffic_live": traffic_live,
            "flop_per_launch": round(flop_per_launch, 1),
            "avg_launch_ms": round(march_avg_ms, 5),
            "launches": int(prof["march_launches"]),
            "flop_basis": "(ray-steps + shade evals the launch counted) x 14,592 FLOP / mean k_trace launch "
                          "duration (per-launch HIP events on the context stream), rank 0",
            "per_rank_frac": [round(float(x) / peak, 4) for x in roof_all[:, 0]] if world > 1 else None,
        },
        "cpu_baseline": None,
    }
    if world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(size, a.max_steps, a.cpu_threads, geometry, matcap, iv, nm)
    print(json.dumps(out), file=jout, flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
