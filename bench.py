#!/usr/bin/env python3
"""bench.py — ed25519 verifies/s on MI355X for the Tendermint commit-verification hot path.

Metric (BASELINE.json): "ed25519 verifies/sec at 1/8 MI355X".  Workload: configs[1],
"Raw batch of 1M random ed25519 signatures (~120-byte canonical vote sign-bytes)
on one MI355X" — SURVEY.md §8d C2: 1,048,576 signatures per GPU, each with its
own key (no key reuse: the generic, worst-case path), CanonicalVote sign-bytes
messages.  A step = one verification pass over the whole batch, inputs resident
in HBM (host->device copies are outside the timed region; DESIGN.md gives the
PCIe-inclusive rate).  At N GPUs every rank verifies its own 1M batch (weak
scaling, no data-path collective); the per-rank valid counts are summed with one
int64 all-reduce after the timed region (the tally exchange of SURVEY.md §8e).

Extra JSON fields:
  roofline      integer-VALU roofline of the verify kernel (HBM traffic ~212 B/verify
                is negligible; MFMA has no 32x32->64 integer path): achieved
                v_mad_i64_i32 per second = verifies/s(kernel time) x mads/verify,
                against the measured device peak of that instruction.
  cpu_baseline  the C restatement of Go 1.18 crypto/ed25519.Verify (oracle/ed25519_port.c,
                "port"), single thread (the reference verifies on one goroutine), timed on
                a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tendermint-fork_amd"))

# v_mad_i64_i32 per verification of the generic (no key cache) kernel, counted from its
# formulas (DESIGN.md "Roofline"); field mul = 100 mads, square = 55 (radix 2^25.5).
MUL, SQ = 100, 55
# Straus per byte of the scalars: 8 dbl (32 S + 26 M) + 2 cached (-A) adds with their conversions
# (14 M), plus, where a B window ends, p1p1->p3 + niels add + p1p1->p2 instead of one p1p1->p2 (+7 M)
MAIN_VARIANT = int(os.environ.get("TMED_MAIN_WAVES", "6"))
B_WINDOWS = 16 if MAIN_VARIANT == 5 else 32     # radix-2^16 (default) or radix-256 B windows
MADS_STRAUS = 32 * (32 * SQ + 40 * MUL) + B_WINDOWS * 7 * MUL
MADS_TABLE = 64 * MUL                        # 1..8 x (-A), cached form
MADS_DECODE = 255 * SQ + 21 * MUL + MUL      # Point.SetBytes (sqrt-ratio chain) + T = XY
# batched finish: one inversion (254 sq + 11 mul) per group of 16 + 3 mul (prefix, 1/Z_j,
# running inverse) + 2 mul (x, y) per signature
MADS_ENCODE = (254 * SQ + 11 * MUL) // 16 + 5 * MUL
MADS_SCALAR = 188                            # mod-L Barrett (v_mad_u64_u32)
MADS_PER_VERIFY_GENERIC = MADS_STRAUS + MADS_TABLE + MADS_DECODE + MADS_ENCODE + MADS_SCALAR
# the dominant kernel (verify_main_kernel): table + Straus + T = XY of the hand-off
MADS_MAIN = MADS_STRAUS + MADS_TABLE + MUL
MAIN_KERNEL = "verify_main_kernel"
if MAIN_VARIANT == 6:
    # half-size scalars (verify_hs.h, the default): W = 33 radix-16 windows (the usual wave
    # maximum; some waves run 34) of 4 dbl (16 S + 13 M) and two cached adds with their
    # conversions (15 M), 8 B steps of two niels adds (+14 M each), two tables (-A, -sign(d) R)
    # and T = XY of A and R; no finish.  Outside the main kernel: decode of A and strict decode
    # of R, the mod-L work (Barrett + |d| S).  The lattice step (fp64 quotient estimates,
    # ~130 Euclid steps) is not counted in mads.
    HS_W = 33
    MADS_MAIN = (HS_W - 1) * (16 * SQ + 13 * MUL) + HS_W * 15 * MUL + 8 * 14 * MUL + 2 * MADS_TABLE + 2 * MUL
    MADS_PER_VERIFY_GENERIC = MADS_MAIN + 2 * MADS_DECODE + MADS_SCALAR + 64 + 188
    MAIN_KERNEL = "verify_main_hs_kernel"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=1 << 20, help="signatures per GPU")
    ap.add_argument("--cpu-sample", type=int, default=150_000, help="signatures timed on the CPU baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-peak", action="store_true")
    ap.add_argument("--mix", choices=["c2", "c5"], default="c2",
                    help="c5: 1%% of the batch replaced by edge-case / invalid tuples (BASELINE C5)")
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from tmed import Engine, lib
    from tmed.workload import c2_messages, c2_seeds

    from tmed.launch import dist_setup
    world, rank, local_rank, dev, coll = dist_setup()
    eng = Engine(local_rank)
    n = args.n

    # ---- synthetic workload (untimed): shard [rank*n, (rank+1)*n) of the C2 stream
    t_gen = time.time()
    start = rank * n
    seeds = c2_seeds(start, n)
    msgs, offs = c2_messages(start, n)
    d_seed = torch.from_numpy(seeds).to(dev)
    d_msg = torch.from_numpy(np.concatenate([msgs, np.zeros(16, np.uint8)])).to(dev)
    d_off = torch.from_numpy(offs.view(np.int32)).to(dev)
    d_sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    d_pub = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    d_out = torch.zeros(n, dtype=torch.uint8, device=dev)
    # a dedicated (non-null) stream: the kernels and the timing events share it
    torch_stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(torch_stream)
    stream = torch_stream.cuda_stream
    eng.sign_device(d_seed, d_msg, d_off, d_sig, d_pub, n, stream)
    torch.cuda.synchronize(dev)
    n_adv = 0
    if args.mix == "c5":
        from tmed.workload import c5_mix
        hp, hs = d_pub.cpu().numpy(), d_sig.cpu().numpy()
        n_adv = len(c5_mix(hp, hs, seed=0x5EED + rank))
        d_pub.copy_(torch.from_numpy(hp))
        d_sig.copy_(torch.from_numpy(hs))
        torch.cuda.synchronize(dev)
    t_gen = time.time() - t_gen

    def step():
        eng.verify_device(d_pub, d_sig, d_msg, d_off, d_out, n, stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ok_first = int(d_out.sum().item())

    # ---- timed region: K steps between barrier + synchronize
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        evs[i][0].record()
        step()
        evs[i][1].record()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    valid = int(d_out.sum().item())
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        tally = torch.tensor([valid, n], dtype=torch.int64, device=coll)
        dist.all_reduce(tally)  # int64 tally all-reduce
        valid_all, n_all = int(tally[0].item()), int(tally[1].item())
    else:
        valid_all, n_all = valid, n
    total = n_all * args.steps
    value = total / elapsed

    result = None
    if rank == 0:
        verifies_per_s_kernel = n / (kernel_ms * 1e-3)
        roof = None
        if not args.no_peak:
            import ctypes
            l = lib()
            l.tmed_valu_peak.restype = ctypes.c_int
            l.tmed_valu_peak.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
            g = ctypes.c_double(0)
            rc = l.tmed_valu_peak(eng._h, 0, ctypes.byref(g))
            peak = g.value / 1e3 if rc == 0 else None  # Tmad/s
            # live per-kernel HIP-event timing of the dominant kernel, one extra (untimed) pass
            eng.set_kernel_timing(True)
            step()
            torch.cuda.synchronize(dev)
            (prep_ms, main_ms, fin_ms), (prep_launches, launches, fin_launches) = eng.kernel_times()
            eng.set_kernel_timing(False)
            achieved = n * MADS_MAIN / (main_ms * 1e-3) / 1e12
            traffic, traffic_src = pmc_traffic(n / max(1, launches))
            roof = {"bound": "valu", "kernel": MAIN_KERNEL, "achieved": round(achieved, 3),
                    "peak": round(peak, 3) if peak else None,
                    "unit": "Tmad/s (v_mad_i64_i32 lane-ops; peak = measured sustained rate)",
                    "frac": round(achieved / peak, 4) if peak else None,
                    "traffic": traffic, "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
                    "traffic_source": traffic_src,
                    "mads_per_verify_main": MADS_MAIN, "mads_per_verify_total": MADS_PER_VERIFY_GENERIC,
                    "kernel_avg_ms": round(main_ms / max(1, launches), 4), "launches_per_step": launches,
                    "prep_kernels_ms": round(prep_ms / max(1, launches), 4), "prep_launches": prep_launches,
                    "finish_kernel_ms": round(fin_ms, 4), "finish_launches": fin_launches,
                    "step_kernel_ms": round(kernel_ms, 3),
                    "algorithmic_bytes_per_verify": 32 + 64 + int(offs[-1]) // n + 4 + 1}
        cpu = cpu_all = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(eng, d_pub, d_sig, msgs, offs, min(args.cpu_sample, n), d_out)
            cpu_all = cpu_baseline_threads(d_pub, d_sig, msgs, offs, n, d_out)
        result = {
            "metric": "ed25519 verifies/sec at 1/8 MI355X",
            "value": round(value, 1),
            "unit": "verifies/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 (GF(2^255-19) radix 2^25.5 limbs, int64 accumulate)",
            "data": "synthetic (C2: distinct key per signature, CanonicalVote sign-bytes, GPU RFC 8032 signer%s)"
                    % (", 1% replaced by edge-case/invalid tuples" if n_adv else ""),
            "config": {"workload": ("C5: adversarial mix, %d ed25519 signatures per GPU with %d edge-case/invalid"
                                    % (n, n_adv)) if n_adv else "C2: raw batch of %d ed25519 signatures per GPU" % n,
                       "signatures_per_gpu": n, "avg_msg_bytes": round(int(offs[-1]) / n, 1),
                       "key_cache": False, "parallelism": "shard-per-gpu x%d" % world},
            "valid": valid_all, "checked": n_all, "all_valid": valid_all == n_all and ok_first == n,
            "adversarial_per_gpu": n_adv,
            "roofline": roof,
            "cpu_baseline": cpu,
            "cpu_baseline_all_cores": cpu_all,
            "setup_s": round(t_gen, 2),
        }
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    eng.close()
    return result


def pmc_traffic(sigs_per_launch):
    """HBM bytes per main-kernel launch from the committed rocprofv3 --pmc summary
    (tools/pmc_summary.py: FETCH_SIZE x2 + WRITE_SIZE per signature, gfx950-corrected),
    scaled to this run's launch size; (None, None) when no summary is present."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as fh:
            pmc = json.load(fh)
    except (OSError, ValueError):
        return None, None
    for k, d in pmc.items():
        if k.split("<")[0] == MAIN_KERNEL and "hbm_bytes_per_sig" in d:
            return round(d["hbm_bytes_per_sig"] * sigs_per_launch), "profiles/pmc_summary.json[%s]" % k
    return None, None


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline_threads(d_pub, d_sig, msgs, offs, m, d_out):
    """The same port on one GPU's share of the host (16 threads, or fewer cores): the
    embarrassingly parallel upper bound SURVEY.md §8d asks for beside the 1-core figure."""
    sys.path.insert(0, ROOT)
    from oracle import port  # cpu_baseline leg only
    nt = min(16, os.cpu_count() or 1)
    pubs = d_pub[:m].cpu().numpy()
    sigs = d_sig[:m].cpu().numpy()
    o = offs[: m + 1].astype(np.uint64)
    t = time.perf_counter()
    out = port.verify_batch(pubs, sigs, msgs, o, nthreads=nt)
    dt = time.perf_counter() - t
    return {"value": round(m / dt, 1), "unit": "verifies/s", "cores": nt, "kind": "port",
            "sample": "all %d signatures of the batch, %d threads, %.1f s; %s; host cpu_count=%d"
                      % (m, nt, dt, _cpu_model(), os.cpu_count() or 1),
            "gpu_decisions_match": bool((d_out[:m].cpu().numpy() == out).all())}


def cpu_baseline(eng, d_pub, d_sig, msgs, offs, m, d_out):
    """Single-thread C restatement of the Go verify on the first m tuples (oracle/ed25519_port.c);
    its decisions are also compared with the GPU's on that sample."""
    sys.path.insert(0, ROOT)
    from oracle import port  # cpu_baseline leg only
    pubs = d_pub[:m].cpu().numpy()
    sigs = d_sig[:m].cpu().numpy()
    o = offs[: m + 1].astype(np.uint64)
    t = time.perf_counter()
    out = port.verify_batch(pubs, sigs, msgs, o, nthreads=1)
    dt = time.perf_counter() - t
    ncores = os.cpu_count() or 1
    gpu = d_out[:m].cpu().numpy()
    return {"value": round(m / dt, 1), "unit": "verifies/s", "cores": 1, "kind": "port",
            "sample": "first %d signatures of the same batch, 1 thread, %.1f s; valid=%d; host cpu_count=%d"
                      % (m, dt, int(out.sum()), ncores),
            "gpu_decisions_match": bool((gpu == out).all())}


if __name__ == "__main__":
    main()
