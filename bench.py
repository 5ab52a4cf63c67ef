#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric on MI355X.

Metric: Msamples/s resampled (float32, 44.1k->48k QualityHigh) + RMS error vs
the reference (oracle).  Workload (BASELINE configs[1]): one stereo float32
stream of 600 s (26,460,000 frames) per GPU, 44.1 kHz -> 48 kHz through
resampler.New with QualityHigh (engine.Quality24Bit), inputs resident in HBM.
One step = Reset + Process(whole stream) + Flush, i.e. the complete job; the
ProcessInto chunking of the reference does not change any output value
(constant.go:270-276), so the stream goes through in one call.

N>1 GPUs: one process per GPU (torchrun), every rank resamples its own
independent stereo stream (weak scaling, streams sharded, no data-path
collective); RCCL (torch.distributed nccl) only all-reduces the timing and
sample counters after the timed region.  value = all input samples of all
ranks / max-over-ranks wall time.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-audio-resampler_amd")]

import numpy as np  # noqa: E402

METRIC = "Msamples/s resampled (float32, 44.1k→48k QualityHigh) + RMS error vs Go ref"
IN_RATE, OUT_RATE, CHANNELS = 44100, 48000, 2
# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md, chip-level table)
PEAK_F32_MATRIX_TFLOPS = 157.3
PEAK_F16_MATRIX_TFLOPS = 2500.0  # dense
PEAK_HBM_GBPS = 8000.0
# reference-algorithm flops per input sample (cfg2)
REF_ALGO_FLOPS_PER_SAMPLE = 1017.6


def synth_stream(frames, channels, seed, rate=IN_RATE):
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


def cpu_baseline(target_s=12.0):
    """The CPU restatement of the reference path (oracle/, 'port') timed on one
    host core: New(44.1k->48k, stereo, QualityHigh) Process+Flush in float64
    (the reference's ProcessFloat32 computes in float64, constant.go:121-146)."""
    from oracle import oracle as O
    O.build()
    probe = 2.0
    frames = int(probe * IN_RATE)
    x = synth_stream(frames, CHANNELS, 4242).astype(np.float64)

    def run(xx):
        r = O.NewResampler(IN_RATE, OUT_RATE, CHANNELS, O.P_HIGH)
        t0 = time.perf_counter()
        for c in range(CHANNELS):
            r.process(xx[:, c], c)
            r.flush(c)
        return time.perf_counter() - t0

    dt = run(x)
    secs = max(probe, min(600.0, probe * target_s / max(dt, 1e-3)))
    frames = int(secs * IN_RATE)
    x = synth_stream(frames, CHANNELS, 4242).astype(np.float64)
    dt = run(x)
    return {"value": round(frames * CHANNELS / dt / 1e6, 3), "unit": "Msamples/s", "cores": 1, "kind": "port",
            "sample": f"{secs:.1f} s of stereo 44.1k->48k QualityHigh (New path, float64 compute), "
                      f"Process+Flush, single thread, {dt:.1f} s wall"}


def load_traffic(workload):
    """HBM bytes per launch of the dominant kernel from the committed PMC run
    (profiles/pmc_<workload>.json written by tools/pmc_traffic.py), else None."""
    p = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--seconds", type=float, default=600.0, help="stream length per GPU (BASELINE cfg2: 600)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--check-seconds", type=float, default=5.0, help="prefix checked against the oracle")
    args = ap.parse_args()

    import torch
    import gar

    world, rank, local = dist_env()
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    frames = int(round(args.seconds * IN_RATE))
    lo, hi = shard_streams(world, rank, world)  # one stereo stream per rank
    x_host = synth_stream(frames, CHANNELS, 4242 + 2 * lo)
    x = torch.from_numpy(x_host).to(dev)

    r = gar.New(gar.Config(IN_RATE, OUT_RATE, CHANNELS, gar.QualityHigh, ComputeDtype=gar.F32, Device=dev.index))
    n_out = gar.lib().gar_device_output_size(r._h, frames)
    r.Reset()
    y = torch.empty((n_out, CHANNELS), dtype=torch.float32, device=dev)
    yf = torch.empty((4096, CHANNELS), dtype=torch.float32, device=dev)

    def step():
        r.Reset()
        r.process_device(x, out=y)
        return r.flush_device(out=yf)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    r.profile(True)
    r.profile_read(0)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tail = step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t1 = time.perf_counter()
    kms, launches = r.profile_read(0)
    r.profile(False)
    n_tail = tail.shape[0]

    local_samples = frames * CHANNELS * args.steps
    elapsed, total_samples = reduce_stats(t1 - t0, local_samples, dev)

    # parity of a prefix against the CPU oracle (rank 0)
    rms = None
    if rank == 0 and args.check_seconds > 0:
        from oracle import oracle as O
        O.build()
        m = int(args.check_seconds * IN_RATE)
        ref = O.NewResampler(IN_RATE, OUT_RATE, CHANNELS, O.P_HIGH)
        got = y.cpu().numpy().astype(np.float64)
        errs = []
        for c in range(CHANNELS):
            want = ref.process(x_host[:m, c].astype(np.float64), c)
            errs.append(np.mean((got[: len(want), c] - want) ** 2))
        rms = float(np.sqrt(np.mean(errs)))

    # roofline of the dominant kernel: the fused DFTx2->polyphase FIR launch of
    # Process (HIP events on the launch stream, inside the library).  The
    # split-f16 kernel (GAR_F32) needs 2*3*MACs of f16 MFMA work per output
    # (40 us at the 2.5 PF dense f16 peak for this workload) and moves the
    # algorithmic bytes once (55 us at 8 TB/s): HBM is the binding roofline.
    geom, _ = gar.design_engine(48000.0, 48000.0 * (OUT_RATE / IN_RATE), gar.Engine24Bit)
    useful_macs = geom.useful_macs_per_output
    outs_per_launch = n_out * CHANNELS
    launch_s = (kms / 1e3) / max(launches, 1)
    workload = "cfg2_stereo_f32_44k1_48k_q24_600s"
    traffic = load_traffic(workload)
    algo_bytes = frames * CHANNELS * 4 + outs_per_launch * 4
    achieved_gbps = algo_bytes / launch_s / 1e9 if launches else None
    split = os.environ.get("GAR_HX", "1") != "0"
    f16_flops = 2.0 * 3 * useful_macs * outs_per_launch  # three f16 products per useful MAC
    f32_flops = 2.0 * useful_macs * outs_per_launch
    line = {
        "metric": METRIC,
        "value": round(total_samples / elapsed / 1e6, 2),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "rms_vs_oracle": rms,
        "config": {
            "workload": workload,
            "description": "BASELINE configs[1]: stereo float32 44.1k->48k QualityHigh (engine Quality24Bit), "
                           "600 s stream per GPU, HBM-resident, one Process+Flush per step",
            "channels": CHANNELS,
            "frames_per_stream": frames,
            "output_frames_per_stream": n_out + n_tail,
            "streams_per_gpu": 1,
            "parallelism": f"independent streams, 1 per GPU x {world}",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved_gbps, 1) if achieved_gbps else None,
            "peak": PEAK_HBM_GBPS,
            "unit": "GB/s",
            "frac": round(achieved_gbps / PEAK_HBM_GBPS, 4) if achieved_gbps else None,
            "traffic": traffic,
            "kernel": ("hx_kernel (fused DFTx2->polyphase banded FIR, f16-split v_mfma_f32_16x16x32_f16, f32 accumulation)"
                       if split else "bg_kernel<float> (exact-f32 v_mfma_f32_16x16x4_f32)"),
            "kernel_ms_per_launch": round(launch_s * 1e3, 4),
            "launches": launches,
            "algo_hbm_bytes_per_launch": algo_bytes,
            "algo_bytes_per_input_sample": round(algo_bytes / (frames * CHANNELS), 3),
            "useful_macs_per_output": round(useful_macs, 2),
            "mfma_tflops": round((f16_flops if split else f32_flops) / launch_s / 1e12, 2) if launches else None,
            "mfma_peak_tflops": PEAK_F16_MATRIX_TFLOPS if split else PEAK_F32_MATRIX_TFLOPS,
            "ref_algo_flops_per_input_sample": REF_ALGO_FLOPS_PER_SAMPLE,
            "ref_equiv_tflops": round(REF_ALGO_FLOPS_PER_SAMPLE * frames * CHANNELS / launch_s / 1e12, 3)
            if launches else None,
        },
        "arith": ("f32 I/O; products as three f16 MFMA terms of 22-bit split operands, f32 accumulation "
                  "(error at the level of exact-f32 arithmetic: rms_vs_oracle)" if split else "exact f32 MFMA"),
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
