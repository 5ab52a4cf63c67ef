#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric on MI355X.

Metric: Msamples/s resampled (input samples summed over channels per second)
+ RMS error vs the reference (oracle/).  Default workload (BASELINE configs[1],
SURVEY.md 8(d) config 2): one stereo float32 stream of 600 s (26,460,000
frames) per GPU, 44.1 kHz -> 48 kHz through resampler.New with QualityHigh
(engine.Quality24Bit), inputs resident in HBM.  One step = Reset + Process
(whole stream, one device call) + Flush, i.e. the complete job; ProcessInto
chunking does not change any output value (constant.go:270-276, checked
bit for bit by tests/test_gpu_parity.py), and the chunked drop-in usage is
timed beside it (`streaming`).

Other workloads (--workload):
  ns256  north_star: 256 ch f32 44.1k->48k QualityHigh, 60 s per GPU
  cfg3   256 ch f32 48k->44.1k QualityVeryHigh, 10 s per GPU
  cfg4   1024 independent stereo streams x 10 s, 44.1k->48k QualityHigh,
         sharded contiguously over the ranks (one NewBatch per rank; total
         work fixed: strong scaling)
  cfg5   8 ch f64 96k->44.1k QualityVeryHigh, 60 s in 4800-frame ProcessInto
         chunks (decimator -> DFTx2 -> polyphase, f64 compute)

N>1 GPUs: one process per GPU (torchrun), no data-path collective; RCCL
(torch.distributed nccl) only reduces the timing and sample counters after
the timed region.  value = all input samples of all ranks / max-over-ranks
wall time.
"""
import argparse
import json
import os
import signal as _signal
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-audio-resampler_amd")]

import numpy as np  # noqa: E402

BASELINE_METRIC = "Msamples/s resampled (float32, 44.1k→48k QualityHigh) + RMS error vs Go ref"
# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md chip table; f64 from SURVEY.md 8(d))
PEAK_HBM_GBPS = 8000.0
PEAK_F16_MATRIX_TFLOPS = 2500.0  # dense
PEAK_F64_MATRIX_TFLOPS = 78.6
# reference-algorithm flops per input sample
REF_ALGO_FLOPS = {"cfg2": 1017.6, "ns256": 1017.6, "cfg4": 1017.6, "cfg3": 1169.0, "cfg5": 1807.6, "poly": None,
                  "quick": None, "pcm16": 1017.6, "cfg2_f64": 1017.6, "ns256_f64": 1017.6}
# New path: preset -> precision -> engine quality (stages.go:54-70, pipeline_builder.go:76-100)
ENGINE_Q = {"High": lambda g: g.Engine24Bit, "VeryHigh": lambda g: g.Engine32Bit, "Quick": lambda g: g.EngineQuick}

WORKLOADS = {
    "cfg2": dict(name="cfg2_stereo_f32_44k1_48k_q24_600s", ir=44100, orr=48000, ch=2, preset="High", seconds=600.0,
                 io="f32", compute="F32", streams=1, scaling="weak", chunk=0,
                 desc="BASELINE configs[1]: stereo float32 44.1k->48k QualityHigh (engine Quality24Bit), 600 s "
                      "stream per GPU, HBM-resident, one Process+Flush per step"),
    "ns256": dict(name="ns256_256ch_f32_44k1_48k_q24_60s", ir=44100, orr=48000, ch=256, preset="High", seconds=60.0,
                  io="f32", compute="F32", streams=1, scaling="weak", chunk=0,
                  desc="north_star: 256-channel float32 44.1k->48k QualityHigh, 60 s per GPU, one Process+Flush"),
    "cfg3": dict(name="cfg3_256ch_f32_48k_44k1_q32_10s", ir=48000, orr=44100, ch=256, preset="VeryHigh", seconds=10.0,
                 io="f32", compute="F32", streams=1, scaling="weak", chunk=0,
                 desc="BASELINE configs[2]: 256-channel float32 48k->44.1k QualityVeryHigh (Quality32Bit), 10 s"),
    "cfg4": dict(name="cfg4_1024x_stereo_f32_44k1_48k_q24_10s", ir=44100, orr=48000, ch=2, preset="High",
                 seconds=10.0, io="f32", compute="F32", streams=1024, scaling="strong", chunk=0,
                 desc="BASELINE configs[3]: 1024 independent stereo float32 streams x 10 s 44.1k->48k QualityHigh, "
                      "sharded contiguously over the ranks, one NewBatch per rank"),
    "cfg5": dict(name="cfg5_8ch_f64_96k_44k1_q32_60s_4800chunks", ir=96000, orr=44100, ch=8, preset="VeryHigh",
                 seconds=60.0, io="f64", compute="F64", streams=1, scaling="weak", chunk=4800,
                 desc="BASELINE configs[4]: 8-channel float64 96k->44.1k QualityVeryHigh multi-stage pipeline "
                      "(decimator x1/2 -> DFT x2 -> polyphase), 60 s streamed in 4800-frame ProcessInto chunks"),
    # the same two geometries at the reference New path's own arithmetic: float64 compute of the
    # float32 streams (constant.go:161-199 converts to float64, runs the float64 engine), f64 I/O so the
    # 1e-12 RMS bar is measurable; f64 MFMA-bound (bg_kernel, v_mfma_f64_16x16x4_f64)
    "cfg2_f64": dict(name="cfg2_f64_stereo_f64_44k1_48k_q24_600s", ir=44100, orr=48000, ch=2, preset="High",
                     seconds=600.0, io="f64", compute="F64", streams=1, scaling="weak", chunk=0,
                     desc="cfg2 geometry computed in float64 (the reference's own arithmetic), f64 I/O, 600 s "
                          "stereo stream per GPU, one Process+Flush"),
    "ns256_f64": dict(name="ns256_f64_256ch_f64_44k1_48k_q24_60s", ir=44100, orr=48000, ch=256, preset="High",
                      seconds=60.0, io="f64", compute="F64", streams=1, scaling="weak", chunk=0,
                      desc="north_star geometry computed in float64 (the reference's own arithmetic), f64 I/O, "
                           "256 ch x 60 s per GPU, one Process+Flush"),
    # x != 0 polyphase (live cubic coefficients, poly_kernel) and QualityQuick (cubic_kernel)
    "poly": dict(name="poly_stereo_f32_16k_44k1_q24_600s", ir=16000, orr=44100, ch=2, preset="High", seconds=600.0,
                 io="f32", compute="F32", streams=1, scaling="weak", chunk=0, kind_bytes={4: 4 * (4 + 2.75625)},
                 desc="stereo float32 16k->44.1k QualityHigh: DFT x2 stage, then DFT x2 + polyphase with a "
                      "fractional step (x != 0, poly_kernel), 600 s, one Process+Flush"),
    "pcm16": dict(name="pcm16_stereo_int16_44k1_48k_q24_600s", ir=44100, orr=48000, ch=2, preset="High", seconds=600.0,
                  io="pcm16", compute="F32", streams=1, scaling="weak", chunk=0,
                  desc="cfg2 geometry on 16-bit integer PCM I/O (resample-wav main.go:444-543 scaling/clamp fused "
                       "into the kernel's loads and stores), 600 s, one Process+Flush"),
    "quick": dict(name="quick_stereo_f32_44k1_48k_600s", ir=44100, orr=48000, ch=2, preset="Quick", seconds=600.0,
                  io="f32", compute="F32", streams=1, scaling="weak", chunk=0, kind_bytes={5: 4 * (1 + 48000 / 44100)},
                  desc="stereo float32 44.1k->48k QualityQuick (CubicStage), 600 s, one Process+Flush"),
}


def metric_for(key, w):
    if key == "cfg2":
        return BASELINE_METRIC
    io = {"f32": "float32", "f64": "float64", "pcm16": "int16 PCM"}[w["io"]]
    return (f"Msamples/s resampled ({io}, {w['ir'] / 1000:g}k→{w['orr'] / 1000:g}k Quality{w['preset']}, "
            f"{w['ch'] * w['streams']} ch) + RMS error vs Go ref")


def synth_stream(frames, channels, seed, rate):
    """0.7 sin(440 Hz) + 0.2 sin(1750 Hz) + 0.1 (U - 0.5) per channel
    (the generator shape of processinto_test.go:19-30), float32 [frames, ch]."""
    out = np.empty((frames, channels), dtype=np.float32)
    t = np.arange(frames, dtype=np.float64) / rate
    for c in range(channels):
        rng = np.random.default_rng(seed + c)
        p1, p2 = rng.random() * 2 * np.pi, rng.random() * 2 * np.pi
        out[:, c] = (0.7 * np.sin(2 * np.pi * 440 * t + p1) + 0.2 * np.sin(2 * np.pi * 1750 * t + p2)
                     + 0.1 * (rng.random(frames) - 0.5))
    return out


def synth_device(torch, frames, channels, seed, rate, dtype):
    """The same signal shape generated on the device (10^9 samples in well under a second)."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    t = torch.arange(frames, device="cuda", dtype=torch.float64) / rate
    ph = torch.rand((2, channels), generator=g, device="cuda", dtype=torch.float64) * 2 * np.pi
    x = torch.empty((frames, channels), device="cuda", dtype=dtype)
    blk = max(1, (1 << 26) // max(channels, 1))
    for s in range(0, frames, blk):
        tt = t[s:s + blk, None]
        noise = torch.rand((tt.shape[0], channels), generator=g, device="cuda", dtype=torch.float64) - 0.5
        x[s:s + blk] = (0.7 * torch.sin(2 * np.pi * 440 * tt + ph[0]) + 0.2 * torch.sin(2 * np.pi * 1750 * tt + ph[1])
                        + 0.1 * noise).to(dtype)
    return x


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def shard_streams(n_streams, rank, world):
    """Contiguous block of independent streams owned by `rank`."""
    base, rem = divmod(n_streams, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def reduce_stats(elapsed_s, samples, device=None):
    """max elapsed and summed samples over ranks (the only collective)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return elapsed_s, samples
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=device)
    s = torch.tensor([float(samples)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    return float(t.item()), float(s.item())


def cpu_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count() or 1
    return model, os.cpu_count(), avail


def cpu_quota():
    """CPUs this process may keep busy: the cgroup CPU quota (cpu.max) if one is set, else None."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                q, p = f.read().split()[:2]
            if q != "max":
                return max(1, int(-(-int(q) // int(p))))
        except (OSError, ValueError):
            pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            p = int(f.read())
        if q > 0:
            return max(1, -(-q // p))
    except (OSError, ValueError):
        pass
    return None


def rank_devices(world, rank, dev, dry):
    """Every rank's process and device (all_gather_object over the process group when world > 1)."""
    import socket
    me = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "host": socket.gethostname(),
          "device": "dry-run (no GPU)" if dry else str(dev)}
    if not dry:
        import torch
        me["device_name"] = torch.cuda.get_device_name(dev)
    if world == 1:
        return [me]
    import torch.distributed as dist
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, me)
    return out


def front_keys(line):
    """The JSON line with the figures a reader (and the driver's parser) needs first: the contract's
    keys, then the dominant kernel's per-launch time and roofline fraction, the streaming-call
    figures and the CPU baseline, flat; everything else after them."""
    roof = line.get("roofline") or {}
    st = (line.get("secondary") or {}).get("stream4096") or {}
    stb = (line.get("secondary") or {}).get("stream4096_batch1024") or {}
    s256 = line.get("streaming_256ch") or {}
    cpu = line.get("cpu_baseline") or {}
    flat = {
        "kernel_ms_per_launch": roof.get("kernel_ms_per_launch"),
        "kernel_ms_min_median_max": roof.get("kernel_ms_min_median_max"),
        "roofline_frac": roof.get("frac"),
        "stream_dev_us_per_call": (st.get("device_api") or {}).get("us_per_call"),
        "stream_host_us_per_call": (st.get("host_cabi") or {}).get("us_per_call"),
        "stream_256ch_host_ms_per_call": s256.get("ms_per_call"),
        "stream_batch1024_dev_us_per_call": (round(stb["ms_per_step"] * 1e3, 2) if stb.get("ms_per_step") else None),
        "stream_batch1024_msamples_per_s": stb.get("value"),
        "cpu_baseline_msamples_per_s": cpu.get("value"),
        "cpu_baseline_cores": cpu.get("cores"),
    }
    head = ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "rms_vs_oracle"]
    out = {k: line[k] for k in head if k in line}
    out.update({k: v for k, v in flat.items() if v is not None})
    out.update({k: v for k, v in line.items() if k not in out})
    return out


def cpu_baseline(w, target_s=10.0):
    """The CPU restatement of the reference path (oracle/, 'port', AVX2 build) timed on
    the host: New(ir->orr, QualityX) Process+Flush per channel in float64 (the
    reference's ProcessFloat32 computes in float64, constant.go:121-146), the
    methodology of throughput_comparison_test.go:102-148.  One core, then every
    core this process may use (one independent stream per thread, like
    EnableParallel's goroutine per channel, constant.go:223-249; the oracle
    releases the GIL inside its C calls)."""
    from oracle import oracle as O
    O.build()
    preset = getattr(O, "P_" + w["preset"].upper())
    ch = min(w["ch"], 2)

    def run(xx):
        r = O.NewResampler(w["ir"], w["orr"], ch, preset)
        t0 = time.perf_counter()
        for c in range(ch):
            r.process(xx[:, c], c)
            r.flush(c)
        return time.perf_counter() - t0

    probe = 1.0
    x = synth_stream(int(probe * w["ir"]), ch, 4242, w["ir"]).astype(np.float64)
    dt = run(x)
    secs = max(probe, min(w["seconds"], probe * target_s / max(dt, 1e-3)))
    frames = int(secs * w["ir"])
    x = synth_stream(frames, ch, 4242, w["ir"]).astype(np.float64)
    dt1 = run(x)
    one = frames * ch / dt1 / 1e6
    model, ncpu, avail = cpu_info()
    quota = cpu_quota()
    # every CPU this process may use (affinity), capped by a cgroup quota if one is set: the
    # reference's EnableParallel runs a goroutine per channel on all cores (constant.go:223-249)
    threads = max(1, min(avail, quota) if quota else avail)
    secs_t = max(probe, min(secs / 2, secs * 8.0 / threads))  # bounded wall time however many threads
    fr_t = int(secs_t * w["ir"])
    xt = x[:fr_t]
    res = [0.0] * threads

    def worker(i):
        res[i] = run(xt)

    ths = [threading.Thread(target=worker, args=(i,)) for i in range(threads)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dtn = time.perf_counter() - t0
    alln = threads * fr_t * ch / dtn / 1e6
    return {"value": round(alln, 3), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"{threads} threads x {secs_t:.1f} s independent {ch}-ch {w['ir']}->{w['orr']} "
                      f"Quality{w['preset']} streams (New path, float64 compute, oracle/ AVX2 build), "
                      f"Process+Flush per channel, {dtn:.1f} s wall",
            "single_core": {"value": round(one, 3), "cores": 1,
                            "sample": f"{secs:.1f} s of the same stream, one thread, {dt1:.1f} s wall"},
            "cpu_model": model, "nproc": ncpu, "cpus_usable": avail, "cgroup_cpu_quota": quota}


def pmc_traffic(args, workload, kernel_keys):
    """HBM bytes per launch of the dominant kernel, measured now: two rocprofv3 PMC
    passes (FETCH_SIZE, then WRITE_SIZE: 3 + 2 TCC counters do not fit one pass)
    over a short child run of this same workload; corrected as
    MI355X_MICROARCH.md's HBM section prescribes (KiB; gfx950 FETCH_SIZE counts
    half the bytes of a wide streaming read -> x2).  None if the profiler is
    unavailable or fails."""
    import csv
    import glob
    prof = "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, "rocprofv3 not found"
    out = {}
    env = dict(os.environ, TMPDIR="/tmp")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="gar_pmc_", dir="/tmp")
        cmd = [prof, "--pmc", counter, "-d", d, "-o", "run", "--output-format", "csv", "--",
               sys.executable, os.path.join(ROOT, "bench.py"), "--workload", workload, "--steps", "2",
               "--warmup", "1", "--no-cpu-baseline", "--check-seconds", "0", "--no-pmc", "--no-streaming",
               "--secondary", "none"]
        try:
            p = subprocess.Popen(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                                 start_new_session=True)
            try:
                p.wait(timeout=180)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, _signal.SIGKILL)
                p.wait()
                return None, f"{counter} pass timed out"
            if p.returncode != 0:
                return None, f"{counter} pass rc {p.returncode}"
        except OSError as e:
            return None, str(e)
        per, grid = {}, {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row.get("Kernel_Name", "")
                    if not any(kk in name for kk in kernel_keys):
                        continue
                    key = (f, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                    per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
                    grid[key] = int(float(row.get("Grid_Size") or 0))
        if not per:
            return None, f"{counter}: no dispatch of {kernel_keys}"
        # the stream-body launch moves the most bytes (a flush tail or a batch's small launches can
        # have the larger grid): average the dispatches within 1 % of the largest count
        vmax = max(per.values())
        vals = [v for v in per.values() if v >= 0.99 * vmax]
        out[counter] = sum(vals) / len(vals)
    corr = FETCH_CORRECTION[LOAD_WIDTH.get(workload, 16)]
    rd = out["FETCH_SIZE"] * 1024 * corr
    wr = out["WRITE_SIZE"] * 1024
    return {"read_bytes": rd, "write_bytes": wr, "bytes": rd + wr, "fetch_correction": corr,
            "read_bytes_uncorrected": out["FETCH_SIZE"] * 1024}, None


# bytes per lane of the dominant kernel's input loads (gar_hxs.hpp hxsRegIssue / gar_hxt.hpp hxtIssue:
# STEREO buffer_load_dwordx2, ROW16 dwordx4, PCM16 stereo dword; cfg5's bg_rt / bg_rb kernels: one 8-B f64
# global load per lane and step for A and B (gar_bg.hpp bg_rb_kernel), each lane of a B load on its
# own 64-B row of the interleaved 8-channel stream -- the x2 streaming calibration is an upper bound
# there, so bench also reports the uncorrected read bytes)
LOAD_WIDTH = {"cfg2": 8, "cfg4": 8, "ns256": 16, "cfg3": 16, "pcm16": 4, "cfg5": 8, "poly": 4, "quick": 4,
              "cfg2_f64": 4, "ns256_f64": 4}  # bg_kernel: LDS-DMA global_load_lds_dword, 4 B per lane
KIND_NAMES = {0: "fused DFTx2->polyphase FIR", 1: "DFT FIR", 2: "decimator FIR", 3: "fused FIR (flush)",
              4: "polyphase with live cubic coefficients (poly_kernel)", 5: "QualityQuick cubic stage (cubic_kernel)"}
# profile kind -> engine kind of the stage it runs (gar_engine_geometry.kind: 1 DFT-only, 2 DFT+poly, 3 decim, 0 cubic)
KIND_STAGE = {0: (2,), 1: (1, 2), 2: (3,), 4: (2,), 5: (0,)}
# gfx950 FETCH_SIZE under-count per load width: MI355X_MICROARCH.md's HBM section gives x2 for
# 16-B/lane streaming reads; calibrated here on 1 GiB read once with buffer_load_dwordx4/x2/dword
# (tools/ubench/fetch_calib.hip, profiles/r03_fetch_calib.txt): FETCH_SIZE = 0.500 of the bytes at
# 16, 8 and 4 B/lane; WRITE_SIZE = 1.000 at 16 and 8 B/lane
FETCH_CORRECTION = {16: 2.0, 8: 2.0, 4: 2.0}


def secondary_default(primary, world):
    """Workloads timed beside the primary line (each with its own ms, roofline and PMC traffic):
    the north-star 256-ch stream, BASELINE configs[2], configs[4], the cfg2 / north-star geometries
    at the reference's float64 arithmetic and -- the scaling config, at every world size -- configs[3]."""
    if primary != "cfg2":
        return []
    return ["ns256", "cfg3", "cfg5", "cfg4", "cfg2_f64", "ns256_f64"] if world == 1 else ["cfg4"]


def run_workload(key, args, steps, warmup, world, rank, dev, primary):
    """Time `steps` steps (after `warmup`) of workload `key` on this rank; returns its JSON
    object (value = all ranks' input samples / max-over-ranks wall time) and the dominant
    kernel's rocprof name keys."""
    import gar
    w = dict(WORKLOADS[key])
    if primary and args.seconds:
        w["seconds"] = args.seconds
    dry = args.dry_run
    torch = None
    if not dry:
        import torch
    frames = int(round(w["seconds"] * w["ir"]))
    if w["scaling"] == "strong":
        s_lo, s_hi = shard_streams(w["streams"], rank, world)
    else:
        s_lo, s_hi = rank, rank + 1  # one stream (batch) per rank
    n_streams = s_hi - s_lo
    C = w["ch"] * (n_streams if w["scaling"] == "strong" else 1)
    pcm_scale = 1.0 / 32767.0 if w["io"] == "pcm16" else None  # main.go:54, :449-460
    x_host = None
    x = None
    if not dry:
        tdt = {"f32": torch.float32, "f64": torch.float64, "pcm16": torch.int16}[w["io"]]
        if key == "cfg2":  # the exact generator of the round-1 line (numpy, per-channel seeds)
            x_host = synth_stream(frames, C, 4242 + 2 * s_lo, w["ir"])
            x = torch.from_numpy(x_host).to(dev)
        elif pcm_scale:
            xs = synth_device(torch, frames, C, 4242 + 7919 * s_lo, w["ir"], torch.float32)
            x = torch.round(xs.clamp(-1, 1) * (32767 * 0.98)).to(torch.int16)
            del xs
        else:
            x = synth_device(torch, frames, C, 4242 + 7919 * s_lo, w["ir"], tdt)

    q = getattr(gar, "Quality" + w["preset"])
    cd = getattr(gar, w["compute"])
    didx = dev.index if dev is not None else 0
    if w["scaling"] == "strong":
        r = gar.NewBatch(gar.Config(w["ir"], w["orr"], w["ch"], q, ComputeDtype=cd, Device=didx, DryRun=dry), n_streams)
    else:
        r = gar.New(gar.Config(w["ir"], w["orr"], C, q, ComputeDtype=cd, Device=didx, DryRun=dry))
    chunk = w["chunk"]
    bounds = [(s, min(chunk, frames - s)) for s in range(0, frames, chunk)] if chunk else [(0, frames)]
    L = gar.lib()
    if dry:
        import ctypes as Ct
        io = {"f32": gar.F32, "f64": gar.F64, "pcm16": gar.PCM16}[w["io"]]
        nz = Ct.c_void_p(1)  # never dereferenced by a dry-run handle

        def step():  # the host state machine only (no device work): exact per-call output counts
            r.Reset()
            o = 0
            got = Ct.c_int64(0)
            for _, n in bounds:
                gar._check(L.gar_process_device(r._h, nz, io, C, 1, n, C, nz, io, C, 1, 1 << 40, Ct.byref(got), None))
                o += got.value
            gar._check(L.gar_flush_device(r._h, C, nz, io, C, 1, 1 << 40, Ct.byref(got), None))
            return o, got.value
    else:
        # output bound: the exact total depends on the carried phase, so allocate ratio*frames + slack
        n_out = int(frames * w["orr"] / w["ir"]) + 64 * (len(bounds) + 1)
        y = torch.empty((n_out, C), dtype=tdt, device=dev)
        yf = torch.empty((max(L.gar_device_flush_size(r._h), 1) + 4096, C), dtype=tdt, device=dev)

        def step():
            r.Reset()
            o = 0
            for s, n in bounds:
                o += r.process_device(x[s:s + n], out=y[o:]).shape[0]
            tail = r.flush_device(out=yf)
            return o, tail.shape[0]

    def sync():
        if not dry:
            torch.cuda.synchronize()

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    # Kernel timing: HIP events around every launch, inside the timed region for one-launch steps
    # (they agree with rocprof there); chunked workloads (hundreds of launches per step) take them in
    # a separate pass after the timed steps, so the timed steps carry no event packets.
    inline_prof = os.environ.get("GAR_BENCH_PROF_INLINE", "0" if w["chunk"] else "1") == "1" and not dry
    for _ in range(warmup):
        step()
    sync()
    if inline_prof:  # HIP events around the FIR launches inside the timed region (on the launch stream);
        # not around the flush (kind 3, never the dominant kernel): each event pair costs stream time
        r.profile(True, kinds=(0, 1, 2, 4, 5))
        for k in range(6):
            r.profile_read(k)
    barrier()
    sync()
    # inline events on every EVENT_EVERY-th step only: an event pair costs a few us of stream time (r05f
    # trace), so the steps between them run as a caller's would; the kernel average is over the
    # bracketed launches
    every = int(os.environ.get("GAR_BENCH_EVENT_EVERY", "4"))
    t0 = time.perf_counter()
    for k in range(steps):
        if inline_prof:
            L.gar_profile_enable(r._h, int(k % every == 0))
        n_proc, n_tail = step()
    sync()
    barrier()
    t1 = time.perf_counter()
    if not dry and not inline_prof:  # a separate profiled pass (the timed steps carry no event packets)
        r.profile(True)
        for k in range(6):
            r.profile_read(k)
        for _ in range(steps):
            step()
        sync()
    prof = {k: (r.profile_read(k) if not dry else (0.0, 0)) for k in range(6)}
    if not dry:
        r.profile(False)

    local_samples = frames * C * steps
    local_ms = (t1 - t0) / steps * 1e3
    elapsed, total_samples = reduce_stats(t1 - t0, local_samples, dev if not dry else None)
    _, total_out = reduce_stats(0.0, (n_proc + n_tail) * C, dev if not dry else None)

    rms, rms_tail = None, None
    check_s = args.check_seconds if primary else min(args.check_seconds, 2.0)
    if rank == 0 and check_s > 0 and not dry:
        rms, rms_tail = oracle_check(w, key, gar, x, x_host, y, yf, n_proc, n_tail, frames, C, check_s, pcm_scale)

    obj = {
        "metric": metric_for(key, w),
        "value": round(total_samples / elapsed / 1e6, 2),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(elapsed / steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": w["scaling"],
        "vs_baseline": None,
        "dtype": w["io"],
        "data": "synthetic",
        "rms_vs_oracle": rms,
        "rms_vs_oracle_tail": rms_tail,
        "config": {
            "workload": w["name"],
            "description": w["desc"],
            "channels": C,
            "frames_per_stream": frames,
            "output_frames_per_stream": n_proc + n_tail,
            "streams_per_gpu": n_streams,
            "chunk_frames": chunk or None,
            "parallelism": (f"{w['streams']} streams sharded over {world} GPUs" if w["scaling"] == "strong"
                            else f"independent streams, 1 per GPU x {world}"),
        },
        "output_samples_total": int(total_out),
        "input_samples_total": int(total_samples / steps),
        "local_ms_per_step": round(local_ms, 4),
    }
    kernel_keys = []
    if not dry:
        roof, kernel_keys = roofline(w, key, gar, r, prof, steps, frames, C, n_proc, n_tail)
        obj["roofline"] = roof
        roof["kernel_timing"] = ((f"HIP events around the launches of every {int(os.environ.get('GAR_BENCH_EVENT_EVERY', '4'))}th "
                                  "timed step, inside the timed region, on the launch stream") if inline_prof
                                 else "HIP events around each launch, in a separate pass after the timed steps")
        obj["arith"] = (("int16 PCM I/O converted in the kernel's loads (float64(i)/32767 -> f32) and stores "
                         "(clamp, x32767, truncate); rms_vs_oracle in full-scale units includes the output "
                         "quantization (~0.6 LSB = 1.8e-5); " if pcm_scale else "f32 I/O; ") +
                        "products as three f16 MFMA terms of 22-bit split operands, f32 accumulation "
                        "(error at the level of exact-f32 arithmetic)" if w["compute"] == "F32"
                        else "f64 I/O and f64 MFMA (v_mfma_f64_16x16x4_f64)")
        if primary and rank == 0 and world == 1 and not args.no_streaming and w["compute"] == "F32" \
                and w["scaling"] == "weak" and w["io"] == "f32":
            obj["streaming"] = time_streaming(gar, torch, w, x, C, dev)
        del x, y, yf
    del r
    if not dry:
        torch.cuda.empty_cache()
    return obj, kernel_keys


def oracle_check(w, key, gar, x, x_host, y, yf, n_proc, n_tail, frames, C, check_s, pcm_scale):
    """Parity vs the CPU oracle (rank 0, after the timed region): a prefix of the first and last
    channels, and a suffix (the last seconds of Process + the whole Flush tail) for single-stage
    fused designs."""
    from oracle import oracle as O
    O.build()
    preset = getattr(O, "P_" + w["preset"].upper())
    m = min(frames, int(check_s * w["ir"]))
    got = y[:n_proc].double().cpu().numpy()
    if pcm_scale:  # PCM: both sides in full-scale units (the oracle is fed the kernel's f32 inputs)
        got = got * pcm_scale

    def xin(a):
        a = np.asarray(a, dtype=np.float64)
        return (a * pcm_scale).astype(np.float32).astype(np.float64) if pcm_scale else a
    chans = sorted({0, C - 1})
    errs = []
    for c in chans:
        xc = xin(x_host[:m, c] if x_host is not None else x[:m, c].cpu().numpy())
        ref = O.NewResampler(w["ir"], w["orr"], 1, preset)
        want = ref.process(xc, 0)
        errs.append(np.mean((got[: len(want), c] - want) ** 2))
    rms = float(np.sqrt(np.mean(errs)))
    rms_tail = None
    # suffix: a single-stage fused design repeats every Qc inputs / Pc outputs, so the oracle
    # restarted at input m0 = k*Qc reproduces outputs k*Pc + j once its transient has passed
    geom, _ = gar.design_engine(48000.0, 48000.0 * (w["orr"] / w["ir"]), ENGINE_Q[w["preset"]](gar))
    stages = O.NewResampler(w["ir"], w["orr"], 1, preset).stages()[1]
    if len(stages) == 1 and geom.fused and w["streams"] == 1:
        Qc, Pc = geom.fir_period_in, geom.fir_period_out
        k = max(0, (frames - m) // Qc)
        m0 = k * Qc
        skip = 4 * geom.fir_taps_max
        tail = yf[:n_tail].double().cpu().numpy() * (pcm_scale or 1.0)
        errs = []
        for c in chans:
            xc = xin(x_host[m0:, c] if x_host is not None else x[m0:, c].cpu().numpy())
            ref = O.NewResampler(w["ir"], w["orr"], 1, preset)
            want = np.concatenate([ref.process(xc, 0), ref.flush(0)])
            full = np.concatenate([got[k * Pc:, c], tail[:, c]])
            if len(full) != len(want):
                errs.append(float("inf"))
                continue
            errs.append(np.mean((full[skip:] - want[skip:]) ** 2))
        rms_tail = float(np.sqrt(np.mean(errs)))
    return rms, rms_tail


def roofline(w, key, gar, r, prof, steps, frames, C, n_proc, n_tail):
    """Roofline object of the dominant kernel kind (HIP events on the launch stream, inside the
    library): algorithmic bytes (HBM-bound f32 FIR) or useful flops (MFMA-bound f64) of the
    stage that kind runs, per launch, over the average launch time."""
    dom = max((0, 1, 2, 4, 5), key=lambda k: prof[k][0])
    kms, launches = prof[dom]
    launch_s = (kms / 1e3) / max(launches, 1)
    per_step = max(launches / steps, 1)
    in_bytes = {"f32": 4, "f64": 8, "pcm16": 2}[w["io"]]
    # the pipeline stage the dominant kind runs, and its input/output samples per step
    nst = r.num_stages()
    geoms = [r.stage_geometry(j) for j in range(nst)]
    sidx = next((j for j in range(nst) if geoms[j][1].kind in KIND_STAGE[dom]), nst - 1)
    ratio_in = 1.0
    for j in range(sidx):
        ratio_in *= geoms[j][0]
    st_ratio, st_geom = geoms[sidx]
    st_in = frames * C * ratio_in
    st_out = (n_proc + n_tail) * C if sidx == nst - 1 else st_in * st_ratio
    if w["compute"] == "F32" and dom in w.get("kind_bytes", {}):
        # that stage's own stream bytes per input frame and channel (its input read once, output written once)
        algo_per_launch = w["kind_bytes"][dom] * frames * C / per_step
        achieved = algo_per_launch / launch_s / 1e9 if launches else None
        roof = {"bound": "hbm", "achieved": round(achieved, 1) if achieved else None, "peak": PEAK_HBM_GBPS,
                "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBPS, 4) if achieved else None}
        kernel_keys = ["poly_kernel"] if dom == 4 else ["cubic_kernel"]
        kname = KIND_NAMES[dom]
        algo_unit_bytes = algo_per_launch
    elif w["compute"] == "F32":
        # HBM-bound streaming FIR: algorithmic bytes = input read once + output written once
        algo_per_launch = (frames * C * in_bytes + n_proc * C * in_bytes) / per_step
        achieved = algo_per_launch / launch_s / 1e9 if launches else None
        roof = {"bound": "hbm", "achieved": round(achieved, 1) if achieved else None, "peak": PEAK_HBM_GBPS,
                "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBPS, 4) if achieved else None}
        kernel_keys = ["hxt_kernel", "hxs_kernel", "hx_kernel"]
        kname = ("hxt_kernel / hxs_kernel / hx_kernel (fused DFTx2->polyphase banded FIR, f16-split "
                 "v_mfma_f32_16x16x32_f16, f32 accumulation)")
        algo_unit_bytes = algo_per_launch
    else:
        # f64: MFMA-bound (f64 matrix rate); useful flops of the dominant stage's own design
        flops_step = 2.0 * st_geom.useful_macs_per_output * st_out
        fl_launch = flops_step / per_step
        achieved = fl_launch / launch_s / 1e12 if launches else None
        roof = {"bound": "mfma", "achieved": round(achieved, 2) if achieved else None,
                "peak": PEAK_F64_MATRIX_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_F64_MATRIX_TFLOPS, 4) if achieved else None}
        chunked = bool(w["chunk"])
        # the kernel that runs the dominant kind: small launches of a chunked stream run the decimator
        # (<= 2 row blocks) on bg_rt_kernel and the composite on bg_rb_kernel (gar_kernels.hip
        # bgSmallGrid); one-shot streams run bg_kernel
        small = "bg_rt_kernel" if dom == 2 else "bg_rb_kernel"
        kernel_keys = (["poly_kernel"] if dom == 4 else [small] if chunked else ["bg_kernel"])
        kern = ('poly_kernel<double>' if dom == 4 else f'{small}<double>' if chunked else 'bg_kernel<double>')
        kname = (f"{kern} ({KIND_NAMES[dom]}, stage {sidx}: {48000:g}->{48000 * st_ratio:g} Hz engine, "
                 "v_mfma_f64_16x16x4_f64)")
        algo_unit_bytes = (st_in * in_bytes + st_out * in_bytes) / per_step
        roof["useful_macs_per_output"] = round(st_geom.useful_macs_per_output, 2)
        roof["stage_outputs_per_step"] = int(st_out)
        if launches:  # the same launch against HBM (its stage's input read once + output written once)
            roof["hbm_gbps"] = round(algo_unit_bytes / launch_s / 1e9, 1)
            roof["hbm_frac"] = round(algo_unit_bytes / launch_s / 1e9 / PEAK_HBM_GBPS, 4)
    roof["ref_algo_flops_per_input_sample"] = REF_ALGO_FLOPS[key]
    roof["kernel_ms_by_kind"] = {KIND_NAMES[k]: round(prof[k][0] / steps, 4) for k in prof if prof[k][1]}
    roof["launches_per_step_by_kind"] = {KIND_NAMES[k]: prof[k][1] / steps for k in prof if prof[k][1]}
    roof.update({"traffic": None, "kernel": kname, "kernel_kind": KIND_NAMES[dom],
                 "kernel_ms_per_launch": round(launch_s * 1e3, 5), "launches": launches})
    try:  # spread of the per-launch event times behind the average
        roof["kernel_ms_min_median_max"] = [round(v, 5) for v in r.profile_launch_stats(dom)]
    except Exception:  # noqa: BLE001 -- an older library without the entry point
        pass
    if algo_unit_bytes:
        roof["algo_hbm_bytes_per_launch"] = int(algo_unit_bytes)
        roof["algo_bytes_per_input_sample"] = round(algo_unit_bytes * per_step / (frames * C), 3)
    if key in ("cfg2", "ns256", "cfg4"):
        geom, _ = gar.design_engine(48000.0, 48000.0 * (w["orr"] / w["ir"]), gar.Engine24Bit)
        useful = geom.useful_macs_per_output
        roof["useful_macs_per_output"] = round(useful, 2)
        outs_launch = n_proc * C / per_step
        roof["mfma_tflops_f16"] = round(2.0 * 3 * useful * outs_launch / launch_s / 1e12, 2) if launches else None
        roof["mfma_peak_tflops_f16"] = PEAK_F16_MATRIX_TFLOPS
    return roof, kernel_keys


def attach_traffic(obj, args, key, kernel_keys):
    """Live PMC traffic of the dominant kernel (world 1); refused when the selected dispatch
    reports fewer bytes than the algorithmic ones (a wrong dispatch or a missed launch)."""
    roof = obj.get("roofline")
    if not roof or not kernel_keys:
        return
    traffic, err = pmc_traffic(args, key, kernel_keys)
    if not traffic:
        roof["traffic_error"] = err
        return
    algo = roof.get("algo_hbm_bytes_per_launch")
    if algo and traffic["bytes"] < 0.9 * algo:
        roof["traffic_error"] = (f"selected dispatch reports {traffic['bytes']:.4g} B < algorithmic {algo:.4g} B "
                                 f"(wrong or missed dispatch): not published")
        roof["traffic_rejected"] = traffic
        return
    roof["traffic"] = traffic["bytes"]
    roof["traffic_read"] = traffic["read_bytes"]
    roof["traffic_write"] = traffic["write_bytes"]
    roof["traffic_fetch_correction"] = traffic["fetch_correction"]
    roof["traffic_read_uncorrected"] = traffic.get("read_bytes_uncorrected")
    if algo:
        roof["traffic_over_algo"] = round(traffic["bytes"] / algo, 4)
        if traffic.get("read_bytes_uncorrected") is not None:
            roof["traffic_over_algo_uncorrected"] = round((traffic["read_bytes_uncorrected"] + traffic["write_bytes"]) / algo, 4)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv):
    """`--gpus N` is authoritative.  Without a torchrun environment and N > 1, start N ranks (one
    process per GPU) as a CHILD `torch.distributed.run` -- before this process touches the GPU --
    and exit with its code; rank 0's JSON line reaches stdout through it.  Under torchrun, a
    WORLD_SIZE that differs from --gpus is an error (a silent 1-rank run would report n_gpus 1).
    Returns the world size this process runs with (or exits)."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is None:
        n = args.gpus if args.gpus is not None else 1
        if n > 1:
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
                   "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + argv
            env = dict(os.environ)
            env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
            env.setdefault("OMP_NUM_THREADS", "1")
            p = subprocess.run(cmd, env=env)
            sys.exit(p.returncode)
        return 1
    if args.gpus is not None and int(ws) != args.gpus:
        sys.stderr.write(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}\n")
        sys.exit(2)
    return int(ws)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of one node; without torchrun, N > 1 starts N ranks itself")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="cfg2", choices=sorted(WORKLOADS))
    ap.add_argument("--seconds", type=float, default=None, help="stream length override (primary workload)")
    ap.add_argument("--secondary", default="auto",
                    help="comma list of workloads timed beside the primary line, 'auto' or 'none'")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=10.0,
                    help="CPU work of the baseline's single-thread sample (bounded; the all-core run is shorter)")
    ap.add_argument("--no-pmc", action="store_true", help="skip the live PMC traffic passes")
    ap.add_argument("--no-streaming", action="store_true", help="skip the chunked drop-in timing")
    ap.add_argument("--check-seconds", type=float, default=5.0, help="prefix (and suffix) checked against the oracle")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: dry-run handles (exact host state machine) over gloo -- the multi-rank "
                         "sharding and reduction end to end on CPU (tests/test_dist.py)")
    args = ap.parse_args()
    launch_ranks(args, sys.argv[1:])

    world, rank, local = dist_env()
    dev = None
    if args.dry_run:
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group(backend="gloo")
    else:
        import torch
        if world > 1:
            import torch.distributed as dist
            torch.cuda.set_device(local)
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
        else:
            torch.cuda.set_device(0)
        dev = torch.device("cuda", torch.cuda.current_device())

    ranks = rank_devices(world, rank, dev, args.dry_run)
    line, keys = run_workload(args.workload, args, args.steps, args.warmup, world, rank, dev, primary=True)
    line["ranks"] = ranks
    line["per_rank"] = per_rank(line, world)
    sec = (secondary_default(args.workload, world) if args.secondary == "auto"
           else [] if args.secondary == "none" else [k for k in args.secondary.split(",") if k])
    if sec:
        line["secondary"] = {}
        for key in sec:
            obj, skeys = run_workload(key, args, min(args.steps, 10), min(args.warmup, 2), world, rank, dev,
                                      primary=False)
            obj["per_rank"] = per_rank(obj, world)
            if rank == 0 and world == 1 and not args.no_pmc and not args.dry_run:
                attach_traffic(obj, args, key, skeys)
            line["secondary"][key] = obj
    # after every timed region and collective: rank 0's own measurements (the other ranks are done)
    # world > 1: a child run on rank 0's GPU of the same per-rank work (weak-scaled workloads only)
    if rank == 0 and not args.no_pmc and not args.dry_run and (world == 1 or WORKLOADS[args.workload]["scaling"] == "weak"):
        attach_traffic(line, args, args.workload, keys)
    if rank == 0 and not args.no_streaming and not args.dry_run and args.workload == "cfg2":
        line.setdefault("secondary", {})
        st = line.pop("streaming", None)
        if st:
            line["secondary"]["stream4096"] = streaming_object(st, WORKLOADS["cfg2"])
        line["streaming_256ch"] = time_streaming_host(WORKLOADS["ns256"], dev)
        line["secondary"]["stream4096_batch1024"] = time_streaming_batch(dev)
    line["cpu_baseline"] = None
    if rank == 0 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(WORKLOADS[args.workload], target_s=args.cpu_baseline_seconds)
    if args.dry_run:
        line["dry_run"] = True
    line["native_lib"] = native_lib_info()
    if rank == 0:
        print(json.dumps(front_keys(line)), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def native_lib_info():
    """Provenance of the HIP library this run loaded: path, size, SHA-256 prefix, mtime, and whether it is
    at least as new as every kernel / host source and the C ABI header it is built from (make's rule)."""
    import hashlib
    pkg = os.path.join(os.path.dirname(os.path.abspath(__file__)), "go-audio-resampler_amd")
    path = os.environ.get("GAR_LIB_PATH") or os.path.join(pkg, "libgar.so")
    if not os.path.exists(path):
        return None
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    srcs = [os.path.join(pkg, "csrc", n) for n in os.listdir(os.path.join(pkg, "csrc"))]
    srcs.append(os.path.join(os.path.dirname(pkg), "include", "gar.h"))
    newest = max(os.path.getmtime(x) for x in srcs)
    mt = os.path.getmtime(path)
    return {"path": os.path.relpath(path, os.path.dirname(pkg)), "bytes": os.path.getsize(path),
            "sha256_16": h.hexdigest()[:16], "mtime_utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(mt)),
            "newer_than_sources": mt >= newest}


def per_rank(obj, world):
    """Every rank's own step time and dominant-kernel events (all_gather_object when world > 1)."""
    roof = obj.get("roofline") or {}
    me = {"rank": int(os.environ.get("RANK", "0")), "local_ms_per_step": obj.get("local_ms_per_step"),
          "kernel_ms_per_launch": roof.get("kernel_ms_per_launch"),
          "kernel_ms_min_median_max": roof.get("kernel_ms_min_median_max"), "launches": roof.get("launches"),
          "frac": roof.get("frac")}
    if world == 1:
        return [me]
    import torch.distributed as dist
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, me)
    return out


def streaming_object(st, w):
    """The 4096-frame drop-in pattern as a workload object of its own (metric / value / ms_per_step =
    one call), device API figures first, the host C-ABI (PCIe-inclusive) beside them."""
    dv = st["device_api"]
    return {"metric": f"Msamples/s resampled (float32, {w['ir'] / 1000:g}k→{w['orr'] / 1000:g}k Quality{w['preset']}, "
                      f"{w['ch']} ch, 4096-frame ProcessInto calls, device API)",
            "value": dv["value"], "unit": "Msamples/s", "ms_per_step": round(dv["us_per_call"] / 1e3, 5),
            "step": "one 4096-frame gar_process_device call", "higher_is_better": True, "dtype": "f32",
            "data": "synthetic", "device_api": dv, "host_cabi": st["host_cabi"], "chunk_frames": st["chunk_frames"]}

def time_streaming(gar, torch, w, x, C, dev, seconds=60.0):
    """The reference's own usage pattern (processinto_bench_test.go:12-205): a stream fed in
    4096-frame ProcessInto calls.  Device API: x already in HBM, one gar_process_device per
    chunk (asynchronous; one synchronise at the end).  Host C-ABI: planar float64 host
    buffers, one gar_process_multi_f64 per chunk (what the cgo shim does: H2D, launches,
    D2H, synchronise inside every call).  Bounded samples of the workload's stream."""
    import ctypes as Ct
    chunk = 4096
    frames = min(x.shape[0], int(seconds * w["ir"]))
    r = gar.New(gar.Config(w["ir"], w["orr"], C, getattr(gar, "Quality" + w["preset"]), ComputeDtype=gar.F32,
                           Device=dev.index))
    y = torch.empty((int(frames * w["orr"] / w["ir"]) + 64 * (frames // chunk + 2), C), dtype=torch.float32,
                    device=dev)
    xs = x[:frames]

    # the C-ABI entry point called per chunk with precomputed arguments (what a cgo / C caller does;
    # Python's tensor slicing and stream lookup per call would be most of a 10 us call)
    L0 = gar.lib()
    st = Ct.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    dt = gar.F32  # float32 device I/O (gar.h GAR_F32)
    es = y.element_size() * C
    ycap = y.shape[0]
    calls_dev = [(Ct.c_void_p(xs[s:].data_ptr()), min(chunk, frames - s)) for s in range(0, frames, chunk)]
    got = Ct.c_int64(0)
    pgot = Ct.byref(got)
    fs_in, cs_in, fs_out, cs_out = xs.stride(0), xs.stride(1), y.stride(0), y.stride(1)
    ybase = y.data_ptr()

    def dev_pass():
        r.Reset()
        o = 0
        for p, n in calls_dev:
            rc = L0.gar_process_device(r._h, p, dt, fs_in, cs_in, n, C, Ct.c_void_p(ybase + o * es), dt, fs_out, cs_out,
                                       ycap - o, pgot, st)
            if rc != 0:
                raise RuntimeError(f"gar_process_device: {rc}")
            o += got.value
        r.flush_device()
        return o

    dev_pass()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dev_pass()
    torch.cuda.synchronize()
    dt_dev = time.perf_counter() - t0
    ncalls = (frames + chunk - 1) // chunk

    # host C-ABI: bounded to `hs` seconds (each call round-trips through PCIe)
    hs = min(seconds / 4, frames / w["ir"])
    hframes = int(hs * w["ir"])
    xh = [np.ascontiguousarray(xs[:hframes, c].double().cpu().numpy()) for c in range(C)]
    rh = gar.New(gar.Config(w["ir"], w["orr"], C, getattr(gar, "Quality" + w["preset"]), ComputeDtype=gar.F32,
                            Device=dev.index))
    cap = int(chunk * w["orr"] / w["ir"]) + 64
    outs = [np.empty(cap) for _ in range(C)]
    outp = (Ct.c_void_p * C)(*[o.ctypes.data for o in outs])
    counts = np.zeros(C, dtype=np.int64)
    L = gar.lib()
    calls = []
    for s in range(0, hframes, chunk):
        n = min(chunk, hframes - s)
        calls.append(((Ct.c_void_p * C)(*[a.ctypes.data + 8 * s for a in xh]), n))

    def host_pass():
        rh.Reset()
        for inp, n in calls:
            st = L.gar_process_multi_f64(rh._h, inp, C, n, outp, cap, counts.ctypes.data)
            if st != 0:
                raise RuntimeError(f"gar_process_multi_f64: {st}")
        rh.FlushMulti()

    host_pass()
    t0 = time.perf_counter()
    host_pass()
    dt_host = time.perf_counter() - t0
    return {
        "chunk_frames": chunk,
        "device_api": {"value": round(frames * C / dt_dev / 1e6, 2), "unit": "Msamples/s", "calls": ncalls,
                       "us_per_call": round(dt_dev / ncalls * 1e6, 2),
                       "sample": f"{frames / w['ir']:.0f} s of the stream, gar_process_device per chunk (ctypes, "
                                 "precomputed arguments) + flush, inputs in HBM, one synchronise at the end"},
        "host_cabi": {"value": round(hframes * C / dt_host / 1e6, 2), "unit": "Msamples/s", "calls": len(calls),
                      "us_per_call": round(dt_host / max(len(calls), 1) * 1e6, 2),
                      "sample": f"{hs:.0f} s, gar_process_multi_f64 per chunk from planar float64 host buffers "
                                "(H2D + launches + D2H + synchronise per call, PCIe-inclusive)"},
    }


def time_streaming_batch(dev, streams=1024, seconds=10.0, chunk=4096):
    """The reference's call size on the shape where the GPU pays: `streams` independent stereo
    44.1k->48k QualityHigh streams (one NewBatch, BASELINE configs[3]'s streams) fed together in
    4096-frame ProcessInto calls through the device API (one launch per call for all streams), inputs
    in HBM, one synchronise at the end (processinto_bench_test.go:12-205's chunk size,
    constant.go:223-249's independent channels)."""
    import ctypes as Ct
    import gar
    import torch
    w = WORKLOADS["cfg4"]
    C = 2 * streams
    frames = int(seconds * w["ir"])
    x = synth_device(torch, frames, C, 777, w["ir"], torch.float32)
    r = gar.NewBatch(gar.Config(w["ir"], w["orr"], 2, gar.QualityHigh, ComputeDtype=gar.F32, Device=dev.index), streams)
    y = torch.empty((int(frames * w["orr"] / w["ir"]) + 64 * (frames // chunk + 2), C), dtype=torch.float32, device=dev)
    L = gar.lib()
    st = Ct.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    es = y.element_size() * C
    calls = [(Ct.c_void_p(x[s:].data_ptr()), min(chunk, frames - s)) for s in range(0, frames, chunk)]
    got = Ct.c_int64(0)
    pgot = Ct.byref(got)

    def dev_pass():
        r.Reset()
        o = 0
        for p, n in calls:
            rc = L.gar_process_device(r._h, p, gar.F32, x.stride(0), x.stride(1), n, C, Ct.c_void_p(y.data_ptr() + o * es),
                                      gar.F32, y.stride(0), y.stride(1), y.shape[0] - o, pgot, st)
            if rc != 0:
                raise RuntimeError(f"gar_process_device: {rc}")
            o += got.value
        r.flush_device()
        return o

    dev_pass()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dev_pass()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out = {"metric": f"Msamples/s resampled (float32, 44.1k→48k QualityHigh, {streams} stereo streams, 4096-frame "
                     "ProcessInto calls, device API)",
           "value": round(frames * C / dt / 1e6, 2), "unit": "Msamples/s", "ms_per_step": round(dt / len(calls) * 1e3, 5),
           "step": f"one 4096-frame gar_process_device call of a {streams}-stream NewBatch ({C} channels)",
           "higher_is_better": True, "dtype": "f32", "data": "synthetic", "calls": len(calls), "streams": streams,
           "sample": f"{seconds:g} s per stream, {len(calls)} calls + flush, inputs in HBM, one synchronise at the end"}
    del x, y, r
    torch.cuda.empty_cache()
    return out


def time_streaming_host(w, dev, calls=40, chunk=4096):
    """The 256-channel drop-in call of the north-star geometry through the host C-ABI: one
    gar_process_multi_f64 per 4096-frame chunk from planar float64 host buffers (H2D + launch +
    D2H + synchronise inside every call, what a cgo caller of ProcessMulti gets), after a warm-up
    pass.  Bounded sample: `calls` calls."""
    import ctypes as Ct
    import gar
    C = w["ch"]
    frames = calls * chunk
    x = synth_stream(frames, C, 99, w["ir"]).astype(np.float64)
    xh = [np.ascontiguousarray(x[:, c]) for c in range(C)]
    r = gar.New(gar.Config(w["ir"], w["orr"], C, getattr(gar, "Quality" + w["preset"]), ComputeDtype=gar.F32,
                           Device=dev.index))
    cap = int(chunk * w["orr"] / w["ir"]) + 64
    outs = [np.empty(cap) for _ in range(C)]
    outp = (Ct.c_void_p * C)(*[o.ctypes.data for o in outs])
    counts = np.zeros(C, dtype=np.int64)
    L = gar.lib()
    args = [((Ct.c_void_p * C)(*[a.ctypes.data + 8 * s for a in xh]), min(chunk, frames - s))
            for s in range(0, frames, chunk)]

    def host_pass():
        r.Reset()
        for inp, n in args:
            st = L.gar_process_multi_f64(r._h, inp, C, n, outp, cap, counts.ctypes.data)
            if st != 0:
                raise RuntimeError(f"gar_process_multi_f64: {st}")

    host_pass()
    passes = []
    for _ in range(5):  # the median pass: one 40-call pass swung by 30 % between boxes (host jitter)
        t0 = time.perf_counter()
        host_pass()
        passes.append(time.perf_counter() - t0)
    dt = sorted(passes)[len(passes) // 2]
    return {"channels": C, "chunk_frames": chunk, "calls": len(args), "ms_per_call": round(dt / len(args) * 1e3, 4),
            "ms_per_call_passes": [round(t / len(args) * 1e3, 4) for t in passes],
            "value": round(frames * C / dt / 1e6, 2), "unit": "Msamples/s",
            "sample": f"median of 5 passes of {len(args)} calls of {chunk} frames x {C} ch {w['ir']}->{w['orr']} "
                      f"Quality{w['preset']}, gar_process_multi_f64 from planar float64 host buffers (PCIe-inclusive)"}


if __name__ == "__main__":
    main()
