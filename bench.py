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
                a bounded sample of the same workload; beside it OpenSSL 3 EVP_DigestVerify
                (anchor_openssl), an independent implementation, on the same sample.
  c2_keyset_variant    the second C2 variant: 10k reused keys, key cache on.
  c1_verifycommit_p50  the metric's second half: VerifyCommit p50 latency @175 validators
                through the seam with the key-set cache as the drop-in uses it (steady state: cache
                hit), the first call after a set change, the cache off, an explicit handle; 1-thread
                CPU baseline beside it.
  c5_adversarial       C5: the C2 batch with 1% invalid signatures of every failure class
                (tmed.workload.c5_mix), rate and mismatches against the port's bits.
  c4_shard             C4 (blocksync, 12,500 blocks x 10,000 validators per GPU = 100k blocks over 8 GPUs) through
                the commit seam, on EVERY rank: contiguous block ranges per rank, the int64 tally
                all-reduce and the per-block decision bitmap all-gather (RCCL at N > 1), MAX of the
                ranks' seam times; verifies/s, outcome mismatches against known answers, the
                per-rank host phase split and the window marshalling beside it.
  c3_light_client      C3 (10k headers x 175 validators, the set changing one key per height) through the
                seam with the key-set cache: headers/s direct (Trusting + Light per header) and by
                bisection (verifySkipping), Got/Needed checked, marshalling beside it (rank 0, N = 1).
  zip215_batch_mode    the OPT-IN ZIP-215 rule (tmed_verify_batch_zip215): C2 all valid (one
                randomized batch equation per 2^20 chunk) and the C5 mix (bisection + exact
                single checks), each against the port's ZIP-215 bits, with the call's statistics.
`--gpus N` without a torchrun environment starts N ranks itself (a child torch.distributed.run).
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
MAIN_VARIANT = 5 if os.environ.get("TMED_MAIN_WAVES") == "5" else 6  # tmed_init reads the same knob
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
    # half-size scalars (verify_hs.h, the default): W = 32 radix-16 windows (the usual wave
    # maximum; some waves run 33) of 4 dbl (16 S + 13 M) and two cached adds with their
    # conversions (15 M), 5 B steps of two niels adds (+14 M each; radix-2^26 tables, 8 steps at
    # radix 2^16 — mads_main_hs), two tables (-A, -sign(d) R)
    # and T = XY of A and R; no finish.  Outside the main kernel: decode of A and strict decode
    # of R, the mod-L work (Barrett + |d| S).  The lattice step (fp64 quotient estimates,
    # ~130 Euclid steps) is not counted in mads.
    # tables by build_table_affine: 2d*xy (1 M) + 7 x (mixed add 3 M + p1p1->p3 4 M + 2dT 1 M)
    MADS_TABLE_HS = 57 * MUL
    HS_W = 32  # the tight window count's usual wave maximum (33 on ~9 % of the waves)
    MADS_MAIN = (HS_W - 1) * (16 * SQ + 13 * MUL) + HS_W * 15 * MUL + 9 * MUL + 5 * 14 * MUL + 2 * MADS_TABLE_HS + 2 * MUL
    MADS_PER_VERIFY_GENERIC = MADS_MAIN + 2 * MADS_DECODE + MADS_SCALAR + 64 + 188
    MAIN_KERNEL = "verify_main_hs_kernel"
# key-cached main kernel (C2 variant, kernels.hip keyset_straus_b24 / keyset_straus_pf): 32 rows of the
# key's radix-256 comb and 11 of the shared radix-2^24 comb of B (16 of the radix-2^16 comb without
# it); the first row is converted niels -> extended (1 M), the middle ones are mixed additions (3 M)
# + p1p1 -> p3 (4 M), the last stops at projective (3 M + 3 M)


def mads_keyset_main(b_bits: int = 24, a_bits: int = 8) -> int:
    """Field products of the key-cached main kernel per signature, in mads: one comb row per
    window (21 with the radix-2^12 -A comb, 23 with radix 2^11, 32 with radix 256; 11 B rows with the
    radix-2^24 B comb, 16 with the radix-2^16 one); the first row is a conversion (1 M), the
    last stops at projective (6 M), the rest are mixed additions (7 M)."""
    rows = {8: 32, 10: 25, 11: 23, 12: 21}[a_bits] + (11 if b_bits == 24 else 16)
    return (1 + (rows - 2) * 7 + 6) * MUL


MADS_KEYSET_MAIN = mads_keyset_main(16)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs of this node; without a torchrun environment bench.py starts N ranks itself")
    ap.add_argument("--steps", type=int, default=200)  # ~2 s timed: long enough for an smi busy sample
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--sigs", type=int, default=1 << 20, help="signatures per GPU (C2: 2^20)")
    ap.add_argument("--cpu-sample", type=int, default=150_000, help="signatures timed on the 1-thread CPU baseline")
    ap.add_argument("--openssl-sample", type=int, default=60_000, help="signatures timed on the OpenSSL anchor")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-peak", action="store_true")
    ap.add_argument("--no-c1", action="store_true", help="skip the VerifyCommit p50 @175 validators leg")
    ap.add_argument("--no-keyset", action="store_true", help="skip the 10k-reused-key C2 variant")
    ap.add_argument("--c1-reps", type=int, default=1000)
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 adversarial-mix leg")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 one-GPU-shard blocksync leg")
    ap.add_argument("--no-zip215", action="store_true", help="skip the opt-in ZIP-215 batch-mode leg")
    ap.add_argument("--c4-blocks", type=int, default=12_500, help="C4 shard: blocks per GPU (100k blocks / 8 GPUs)")
    ap.add_argument("--no-c3", action="store_true", help="skip the C3 light-client leg")
    ap.add_argument("--c3-headers", type=int, default=10_000)
    ap.add_argument("--mix", choices=["c2", "c5"], default="c2",
                    help="c5: 1%% of the batch replaced by edge-case / invalid tuples (BASELINE C5)")
    return ap.parse_args()


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` outside torchrun: start N ranks (one process per GPU) with
    torch.distributed.run as a CHILD process — before anything here touches the GPU — and return
    its exit code (the driver's own N>1 command is this same torchrun line)."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def mads_main_hs(w: float, b_bits: int = 26) -> float:
    """v_mad_i64_i32 of verify_main_hs_kernel per signature at a wave loop length of w windows:
    B steps of two niels adds (+14 M each) — five with the radix-2^26 tables, eight with radix 2^16;
    the top window (digits 0..16 since round 5) adds two table entries per scalar: -A's first entry
    converted to extended (1 M) and three cached additions instead of two (+9 M)."""
    b_steps = 5 if b_bits == 26 else 8
    return (w - 1) * (16 * SQ + 13 * MUL) + w * 15 * MUL + 9 * MUL + b_steps * 14 * MUL + 2 * 57 * MUL + 2 * MUL


def window_summary(eng):
    """Loop-length statistics of the last half-size chunk (tmed_window_stats): the lattice step's
    per-signature window count W and the per-wave maximum the main kernel ran (W = 64 = fallback)."""
    try:
        lh, wh = eng.window_stats()
    except AttributeError:  # an older library build (A/B runs through TMED_LIB)
        return None
    nl, nw = int(lh.sum()), int(wh.sum())
    if nl == 0 or nw == 0:
        return None
    ws = np.arange(65)
    return {"lanes": nl, "waves": nw, "lane_W_mean": round(float((lh * ws).sum()) / nl, 3),
            "wave_W_mean": round(float((wh * ws).sum()) / nw, 3),
            "lane_fallback_W64": int(lh[64]), "wave_W64": int(wh[64]),
            "wave_W_hist": {str(w): int(wh[w]) for w in range(65) if wh[w]}}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args.gpus)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world_env), file=sys.stderr)
        return 2
    import torch
    import torch.distributed as dist

    from tmed import Engine
    from tmed.workload import c2_messages, c2_seeds

    from tmed.launch import BINDING, dist_setup, gpu_count_fields
    world, rank, local_rank, dev, coll = dist_setup()
    eng = Engine(local_rank)
    n = args.sigs

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

    # ---- the dominant kernel's roofline, read right after the C2 timed region (rank 0): the
    # lattice step's window statistics of THIS batch (later legs' seam calls reset them) and one
    # extra untimed pass with live per-kernel HIP-event timing
    roof = peak = None
    if rank == 0:
        roof, peak = roofline_leg(eng, step, dev, n, offs, kernel_ms, args.no_peak)

    # ---- C4 on every rank (weak scaling: c4_blocks per GPU, contiguous heights, RCCL tallies)
    c4 = None
    if not args.no_c4:
        c4 = c4_shard(eng, coll, args.c4_blocks, rank, world)

    result = None
    if rank == 0:
        cpu = cpu_all = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(d_pub, d_sig, msgs, offs, min(args.cpu_sample, n), d_out,
                               min(args.openssl_sample, n))
            cpu_all = cpu_baseline_threads(d_pub, d_sig, msgs, offs, n, d_out, cpu["value"], value)
            cpu["gpu_speedup_vs_1_core"] = round(value / cpu["value"], 1)
            cpu["all_cores"] = {"measured_threads": cpu_all["cores"], "measured_value": cpu_all["value"],
                                "extrapolated_cores": cpu_all["box_cpus"],
                                "extrapolated_value": cpu_all["all_cores_extrapolated"]["value"],
                                "gpu_speedup_vs_all_cores": cpu_all["all_cores_extrapolated"]["gpu_speedup"]}
        keyset = None
        if not args.no_keyset and world == 1:
            keyset = c2_keyset(eng, dev, torch_stream, n, args.steps, args.warmup, peak)
        c1 = None
        if not args.no_c1 and world == 1:
            c1 = c1_latency(eng, args.c1_reps, not args.no_cpu_baseline)
        c5 = None
        if not args.no_c5 and world == 1 and args.mix == "c2":
            c5 = c5_leg(eng, dev, torch_stream, d_pub, d_sig, d_msg, d_off, msgs, offs, n, args.steps // 10 + 1)
        zip_leg = None
        if not args.no_zip215 and world == 1 and args.mix == "c2":
            zip_leg = zip215_leg(eng, dev, torch_stream, d_pub, d_sig, d_msg, d_off, msgs, offs, n, args.steps // 10 + 1)
        c3 = None
        if not args.no_c3 and world == 1:
            c3 = c3_leg(eng, args.c3_headers)
        result = {
            "metric": "ed25519 verifies/sec at %d/8 MI355X" % world,
            "value": round(value, 1),
            "unit": "verifies/s",
            **gpu_count_fields(world),
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
            "c2_keyset_variant": keyset,
            "c1_verifycommit_p50": c1,
            "c5": c5,
            "zip215_batch_mode": zip_leg,
            "c4_shard": c4,
            "c3_light_client": c3,
            "setup_s": round(t_gen, 2),
            "host_binding_rank0": dict(BINDING),
        }
        # LAST key: every leg's headline in a few hundred bytes, so the driver's stdout tail (the
        # end of this line) carries them all
        result["legs"] = legs_summary(result)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    eng.close()
    return 0


def legs_summary(r):
    """Compact headline numbers of every leg (M = 1e6 per second; ms = milliseconds p50)."""
    def g(d, *path):
        for k in path:
            if not isinstance(d, dict) or k not in d:
                return None
            d = d[k]
        return d

    def M(x):
        return None if x is None else round(x / 1e6, 2)

    def ms(x):
        return None if x is None else round(x, 4)

    out = {"c2_Mps": M(r["value"]), "c2_ms": r["ms_per_step"],
           "c2_main_frac": g(r, "roofline", "frac"), "prep_ms": g(r, "roofline", "prep_kernels_ms")}
    k = r.get("c2_keyset_variant")
    if k:
        out["c2_keyed"] = {"Mps": M(k["value"]), "ms": k["ms_per_step"], "frac": g(k, "roofline", "frac")}
    c1 = r.get("c1_verifycommit_p50")
    if c1:
        p = c1.get("paths", {})
        out["c1_ms"] = {"hit": ms(g(p, "cache_hit", "p50_ms")), "first": ms(g(p, "first_call_after_set_change", "p50_ms")),
                        "warmed": ms(g(p, "first_call_after_warmed_set_change", "p50_ms")),
                        "off": ms(g(p, "generic_cache_off", "p50_ms")), "cpu": ms(g(c1, "cpu_baseline", "value"))}
    c3 = r.get("c3_light_client")
    if c3:
        out["c3"] = {"hdr_Mps": M(g(c3, "direct", "headers_per_s")),
                     "incl_marshal_Mps": M(g(c3, "direct", "headers_per_s_incl_marshal")),
                     "plan_frac": g(c3, "direct", "phase_share", "plan_frac"),
                     "mismatches": g(c3, "direct", "outcome_mismatches"),
                     "bisect_hdr_Mps": M(g(c3, "bisection", "headers_per_s"))}
    c4 = r.get("c4_shard")
    if c4:
        out["c4"] = {"Mps": M(c4.get("value")), "incl_marshal_Mps": M(c4.get("value_incl_marshal")),
                     "overlapped_Mps": M(c4.get("value_incl_marshal_overlapped")),
                     "mismatches": c4.get("outcome_mismatches")}
    c5 = r.get("c5")
    if c5:
        out["c5"] = {"Mps": M(c5["value"]), "mismatches": c5["mismatches_vs_port"]}
    z = r.get("zip215_batch_mode")
    if z:
        out["zip215"] = {"c2_Mps": M(g(z, "c2", "value")), "c5_Mps": M(g(z, "c5", "value")),
                         "mismatches": (g(z, "c2", "mismatches_vs_port_zip215") or 0)
                         + (g(z, "c5", "mismatches_vs_port_zip215") or 0)}
    cpu = r.get("cpu_baseline")
    if cpu:
        out["cpu"] = {"1thr": cpu["value"], "x1": cpu.get("gpu_speedup_vs_1_core"),
                      "thr": g(cpu, "all_cores", "measured_threads"), "thr_value": g(cpu, "all_cores", "measured_value"),
                      "all_cores": g(cpu, "all_cores", "extrapolated_cores"),
                      "all_value_extrap": g(cpu, "all_cores", "extrapolated_value"),
                      "x_all": g(cpu, "all_cores", "gpu_speedup_vs_all_cores")}
    return out


def roofline_leg(eng, step, dev, n, offs, kernel_ms, no_peak):
    """`roofline` of the dominant kernel (verify_main_hs_kernel): achieved = signatures per launch x
    the kernel's mads at the measured wave-mean window count (tmed_window_stats of the C2 batch just
    timed) / the launch's live HIP-event duration; peak = the v_mad_i64_i32 rate measured now, on
    this device (tmed_valu_peak).  Returns (roofline dict or None, peak Tmad/s or None)."""
    import torch
    wstats = window_summary(eng) if MAIN_VARIANT != 5 else None
    if no_peak:
        return None, None
    import ctypes
    from tmed import lib
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
    try:
        b_bits = eng.b_window_bits()
    except AttributeError:  # an older library build (A/B runs through TMED_LIB)
        b_bits = 16
    mads_main = MADS_MAIN if wstats is None else mads_main_hs(wstats["wave_W_mean"], b_bits)
    achieved = n * mads_main / (main_ms * 1e-3) / 1e12
    traffic, traffic_src = pmc_traffic(n / max(1, launches))
    clk_main, clk_probe = pmc_clock(MAIN_KERNEL), pmc_clock("valu_probe")
    roof = {"bound": "valu", "kernel": MAIN_KERNEL, "achieved": round(achieved, 3),
            "peak": round(peak, 3) if peak else None,
            "unit": "Tmad/s (v_mad_i64_i32 lane-ops; peak = measured sustained rate)",
            "frac": round(achieved / peak, 4) if peak else None,
            "traffic": traffic, "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
            "traffic_source": traffic_src,
            "mads_per_verify_main": round(mads_main), "mads_per_verify_total": MADS_PER_VERIFY_GENERIC,
            "mads_basis": ("wave-mean window count %.3f (tmed_window_stats of the timed C2 batch), radix-2^%d B "
                           "windows" % (wstats["wave_W_mean"], b_bits)) if wstats else "formula (W = %d)" % HS_W,
            "kernel_avg_ms": round(main_ms / max(1, launches), 4), "launches_per_step": launches,
            "prep_kernels_ms": round(prep_ms / max(1, launches), 4), "prep_launches": prep_launches,
            "finish_kernel_ms": round(fin_ms, 4), "finish_launches": fin_launches,
            "step_kernel_ms": round(kernel_ms, 3),
            "algorithmic_bytes_per_verify": 32 + 64 + int(offs[-1]) // n + 4 + 1,
            "window_stats": wstats}
    # figures of the archived PMC pass (not measured in this run): present only when the summary was
    # collected on this tree's kernel sources, and grouped with its tag
    matching, meta = pmc_meta()
    if matching:
        arch = {"source": "profiles/pmc_summary.json", "collected": meta.get("collected"),
                "kernel_src_sha16": meta.get("kernel_src_sha16")}
        if clk_main:
            # effective clocks (GRBM_GUI_ACTIVE / 8 XCDs / dispatch time, one PMC run for both): the
            # main kernel's table traffic costs clock, not bandwidth
            arch["clock_ghz"] = {"main_kernel": clk_main, "valu_peak_probe": clk_probe}
            if peak and clk_probe:
                # the live fraction with the peak scaled to the main kernel's own clock
                arch["frac_at_kernel_clock"] = round(achieved / (peak * clk_main / clk_probe), 4)
        va = pmc_field(MAIN_KERNEL, "valu_active_frac", 4)
        if va is not None:
            # SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES per wave x the kernel's 2 waves per SIMD: ~1 means
            # the SIMD issues a VALU instruction every slot (issue-bound at its instruction mix)
            arch["valu_issue_busy_est"] = {"valu_active_per_wave": va, "waves_per_simd": 2, "busy": round(2 * va, 3)}
        roof["archived_pmc"] = arch
    else:
        roof["archived_pmc"] = {"omitted": "profiles/pmc_summary.json was not collected on this tree's kernel "
                                           "sources (_meta.kernel_src_sha16)", "summary_meta": meta}
    return roof, peak


def c2_keyset(eng, dev, torch_stream, n, steps, warmup, peak):
    """C2's second variant: n signatures by 10,000 validators with the key cache
    on (tmed_verify_batch_keyset_device: [k](-A) from each key's comb, no doublings), inputs in HBM;
    verifies/s over `steps` timed passes and the roofline of its main kernel (HIP events)."""
    import torch
    from tmed.workload import c2_messages, seeds_from_tag
    nk = 10_000
    kseeds = seeds_from_tag(b"tmed-c2k-key", 0, nk)
    rng = np.random.default_rng(7)
    val_idx = rng.integers(0, nk, n).astype(np.uint32)
    msgs, offs = c2_messages(0, n)
    d_seed = torch.from_numpy(kseeds[val_idx]).to(dev)
    d_msg = torch.from_numpy(np.concatenate([msgs, np.zeros(16, np.uint8)])).to(dev)
    d_off = torch.from_numpy(offs.view(np.int32)).to(dev)
    d_sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    d_pub = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    d_out = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_vi = torch.from_numpy(val_idx.view(np.int32)).to(dev)
    st = torch_stream.cuda_stream
    eng.sign_device(d_seed, d_msg, d_off, d_sig, d_pub, n, st)
    torch.cuda.synchronize(dev)
    pubs = np.zeros((nk, 32), np.uint8)
    pubs[val_idx] = d_pub.cpu().numpy()
    del d_seed, d_pub
    t_ks = time.perf_counter()
    ks = eng.keyset_load(pubs)
    t_ks = time.perf_counter() - t_ks

    def step():
        eng.verify_keyset_device(ks, d_vi, d_sig, d_msg, d_off, d_out, n, st)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    ok_first = int(d_out.sum().item())
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    valid = int(d_out.sum().item())
    eng.set_kernel_timing(True)
    step()
    torch.cuda.synchronize(dev)
    (prep_ms, main_ms, fin_ms), (pl, ml, fl) = eng.kernel_times()
    eng.set_kernel_timing(False)
    try:
        kb = eng.keyset_b_window_bits()
    except AttributeError:  # an older library build (A/B runs through TMED_LIB)
        kb = 16
    try:
        ka = eng.keyset_a_window_bits(ks)
    except AttributeError:
        ka = 8
    eng.keyset_free(ks)
    mads_ks = mads_keyset_main(kb, ka)
    achieved = n * mads_ks / (main_ms * 1e-3) / 1e12 if main_ms > 0 else None
    traffic, traffic_src = pmc_traffic(n / max(1, ml), "verify_keyset_main_kernel")
    return {"metric": "ed25519 verifies/sec at 1/8 MI355X, key cache on (C2 variant: 10k reused keys)",
            "value": round(n * steps / dt, 1), "unit": "verifies/s", "steps": steps,
            "ms_per_step": round(dt / steps * 1e3, 3), "all_valid": valid == n and ok_first == n,
            "keyset_build_s": round(t_ks, 3),
            "roofline": {"bound": "valu", "kernel": "verify_keyset_main_kernel",
                         "achieved": round(achieved, 3) if achieved else None,
                         "peak": round(peak, 3) if peak else None, "unit": "Tmad/s",
                         "frac": round(achieved / peak, 4) if (achieved and peak) else None,
                         "traffic": traffic, "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
                         "traffic_source": traffic_src,
                         "mads_per_verify_main": mads_ks, "b_window_bits": kb, "a_window_bits": ka,
                         "visiting_order": "key-grouped (launch_key_order, charged to prep_kernel_ms)",
                         "kernel_avg_ms": round(main_ms / max(1, ml), 4), "launches_per_step": ml,
                         "prep_kernel_ms": round(prep_ms, 4), "finish_kernel_ms": round(fin_ms, 4)},
            "config": {"workload": "C2 variant: %d signatures by %d validators (seeded), key cache on" % (n, nk)}}


def c5_leg(eng, dev, torch_stream, d_pub, d_sig, d_msg, d_off, msgs, offs, n, steps):
    """BASELINE C5 on the C2 batch: 1 % of the tuples replaced (seed 0x5EED) by the SURVEY §8c edge
    classes (R/S/M bit flips, S + L, small-order A and R, non-canonical A with y >= p, R sign
    flips) through the default generic path; verifies/s over `steps` timed passes, and the GPU's
    decisions against the 16-thread C port on ALL n tuples (gate: 0 mismatches)."""
    import torch
    from tmed.workload import c5_mix
    sys.path.insert(0, ROOT)
    from oracle import port  # checker only
    hp, hs = d_pub.cpu().numpy(), d_sig.cpu().numpy()
    idx = c5_mix(hp, hs, seed=0x5EED)
    p5, s5 = torch.from_numpy(hp).to(dev), torch.from_numpy(hs).to(dev)
    o5 = torch.zeros(n, dtype=torch.uint8, device=dev)
    st = torch_stream.cuda_stream
    eng.verify_device(p5, s5, d_msg, d_off, o5, n, st)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.verify_device(p5, s5, d_msg, d_off, o5, n, st)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    gpu = o5.cpu().numpy()
    nt = min(16, os.cpu_count() or 1)
    t = time.perf_counter()
    exp = port.verify_batch(hp, hs, msgs, offs.astype(np.uint64), nthreads=nt)
    t_port = time.perf_counter() - t
    return {"metric": "ed25519 verifies/sec at 1/8 MI355X, C5 adversarial mix", "value": round(n * steps / dt, 1),
            "unit": "verifies/s", "steps": steps, "ms_per_step": round(dt / steps * 1e3, 3),
            "signatures": n, "replaced": int(len(idx)), "valid": int(gpu.sum()), "expected_valid": int(exp.sum()),
            "mismatches_vs_port": int((gpu != exp).sum()),
            "checker": "oracle/ed25519_port.c on all %d tuples, %d threads, %.1f s" % (n, nt, t_port),
            "config": {"workload": "C5: C2 batch with 1%% replaced by edge-case/invalid tuples, seed 0x5EED"}}


def zip215_leg(eng, dev, torch_stream, d_pub, d_sig, d_msg, d_off, msgs, offs, n, steps):
    """The opt-in ZIP-215 mode (tmed_verify_batch_zip215_device; spec/core/encoding.md:52-54), NOT the
    reference's default rule: the C2 batch as one randomized batch equation (GPU Pippenger MSM), and
    the C5 mix (1% edge/invalid: the equation fails, bisection, exact single checks).  verifies/s,
    the engine's equation / single-check counts, and decisions against the C port's ZIP-215 rule
    (oracle/ed25519_port.c port_verify_zip215, 16 threads) on every tuple."""
    import torch
    from tmed import Engine
    from tmed.workload import c5_mix
    sys.path.insert(0, ROOT)
    from oracle import port  # checker only
    st = torch_stream.cuda_stream
    res = {"metric": "ed25519 verifies/sec at 1/8 MI355X, opt-in ZIP-215 batch mode (not the reference rule)",
           "unit": "verifies/s", "rule": "ZIP-215: permissive A/R decoding, S < L, [8](SB - R - kA) = O"}
    nt = min(16, os.cpu_count() or 1)
    hp, hs = d_pub.cpu().numpy(), d_sig.cpu().numpy()
    o = offs.astype(np.uint64)
    for name, mix in (("c2", False), ("c5", True)):
        p, sg = hp, hs
        if mix:
            p, sg = hp.copy(), hs.copy()
            c5_mix(p, sg, seed=0x5EED)
        dp, ds = torch.from_numpy(p).to(dev), torch.from_numpy(sg).to(dev)
        out = torch.zeros(n, dtype=torch.uint8, device=dev)
        eng.verify_zip215_device(dp, ds, d_msg, d_off, out, n, st)
        torch.cuda.synchronize(dev)
        k = steps if not mix else max(1, steps // 4)
        t0 = time.perf_counter()
        for _ in range(k):
            eng.verify_zip215_device(dp, ds, d_msg, d_off, out, n, st)
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        stats = Engine.zip215_stats()
        gpu = out.cpu().numpy()
        exp = port.verify_batch(p, sg, msgs, o, nthreads=nt, zip215=True)
        res[name] = {"value": round(n * k / dt, 1), "ms_per_step": round(dt / k * 1e3, 3), "steps": k,
                     "valid": int(gpu.sum()), "mismatches_vs_port_zip215": int((gpu != exp).sum()),
                     "engine": stats}
        del dp, ds, out
    res["value"] = res["c2"]["value"]
    res["config"] = {"workload": "C2 batch (and the C5 mix) of %d signatures in ZIP-215 batch mode" % n,
                     "checker": "oracle/ed25519_port.c port_verify_zip215 on all tuples, %d threads" % nt}
    return res


def c4_shard(eng, coll, blocks, rank, world):
    """BASELINE C4 (100k blocks / 8 GPUs): `blocks` blocks x 10,000 validators PER RANK, contiguous
    heights, VerifyCommitLight per block through the pipelined blocksync seam (tmed_blocksync_verify)
    with the set passed WITHOUT a key-set handle (the key-set cache builds its keys after the first,
    untimed window); known-answer bad signatures every 97 blocks, every block's outcome checked
    (bench_commits.c4).  At N ranks: int64 tallies all-reduced, the decision bitmaps all-gathered
    (RCCL over xGMI; gloo with TMED_DIST_BACKEND=gloo), value = all verifies / the slowest rank's seam
    time.  Called on every rank."""
    sys.path.insert(0, ROOT)
    import bench_commits
    r = bench_commits.c4(eng, blocks * world, 10_000, rank, world, coll, 1000, 128, corrupt_every=97)
    r["metric"] = ("blocksync replay verifies/s, C4 sharded over %d GPU(s) (VerifyCommitLight per block)" % world
                   if world > 1 else "blocksync replay verifies/s, one GPU's shard of C4 (VerifyCommitLight per block)")
    if os.environ.get("TMED_DIST_BACKEND") == "gloo" and world > 1:
        r["rehearsal"] = "gloo collectives, ranks sharing the GPUs present: not a scaling measurement"
    return r


def c3_leg(eng, headers):
    """BASELINE C3 through the seam with the key-set cache (bench_commits.c3, policy "cache")."""
    sys.path.insert(0, ROOT)
    import bench_commits
    return bench_commits.c3(eng, headers, 2, "cache", runs=5, bisect_gap=150)


def c1_latency(eng, reps, cpu):
    """BASELINE metric, second half: VerifyCommit p50 latency @175 validators through the seam
    (bench_commits.c1: generic and key-cached paths, `reps` repetitions each, 1-thread CPU port
    beside it)."""
    sys.path.insert(0, ROOT)
    import bench_commits
    r = bench_commits.c1(eng, reps, cpu)
    return {k: r[k] for k in ("metric", "unit", "value", "paths", "reps", "config", "cpu_baseline", "speedup_vs_cpu")
            if k in r}


def load_pmc():
    """The committed rocprofv3 --pmc summary (profiles/pmc_summary.json) when it was collected on the
    kernel sources of this tree (its _meta.kernel_src_sha16, tools/pmc_summary.py), else None: counters
    of an older build are not reported beside this run's live figures."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_summary.json")) as fh:
            pmc = json.load(fh)
    except (OSError, ValueError):
        return None
    from tmed.srcdigest import kernel_src_digest
    if pmc.get("_meta", {}).get("kernel_src_sha16") != kernel_src_digest():
        return None
    return pmc


def pmc_meta():
    """(matching, meta) of the committed PMC summary."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_summary.json")) as fh:
            meta = json.load(fh).get("_meta", {})
    except (OSError, ValueError):
        return False, {}
    return load_pmc() is not None, meta


def pmc_traffic(sigs_per_launch, kernel=None):
    """HBM bytes per launch of `kernel` (default: the generic main kernel) from the committed
    rocprofv3 --pmc summary (tools/pmc_summary.py: FETCH_SIZE x2 + WRITE_SIZE per signature,
    gfx950-corrected), scaled to this run's launch size; (None, reason) when no summary of these
    kernel sources is present."""
    kernel = kernel or MAIN_KERNEL
    pmc = load_pmc()
    if pmc is None:
        return None, "no PMC summary of this tree's kernel sources (profiles/pmc_summary.json _meta)"
    for k, d in pmc.items():
        if k.split("<")[0] == kernel and "hbm_bytes_per_sig" in d:
            return round(d["hbm_bytes_per_sig"] * sigs_per_launch), "profiles/pmc_summary.json[%s]" % k
    return None, None


def pmc_field(kernel, key, nd=3):
    """`key` of `kernel` in the committed PMC summary of this tree's kernels, or None."""
    pmc = load_pmc()
    if pmc is None:
        return None
    for k, d in pmc.items():
        if k.split("<")[0] == kernel and key in d:
            return round(d[key], nd)
    return None


def pmc_clock(kernel):
    """Effective clock (GHz) of `kernel` from the committed PMC summary, or None."""
    return pmc_field(kernel, "effective_clock_ghz")


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


HOST_SHARE_THREADS = 16  # one GPU's share of the box's CPUs (the pool's rule for worker pools)


def _cgroup_cpus():
    """The CPU bandwidth this process's cgroup allows, in CPUs (cgroup v2 cpu.max / v1 cfs quota), or
    None when unlimited or unreadable: beside os.cpu_count(), what an all-threads run could use."""
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", lambda t: [t.strip(), None])):
        try:
            with open(path) as fh:
                q, per = parse(fh.read())
        except (OSError, ValueError):
            continue
        if q in ("max", "-1"):
            return None
        if per is None:
            try:
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
                    per = fh.read().strip()
            except OSError:
                return None
        try:
            return round(int(q) / int(per), 2)
        except (ValueError, ZeroDivisionError):
            return None
    return None


def cpu_baseline_threads(d_pub, d_sig, msgs, offs, m, d_out, one_thread_value, gpu_value):
    """The port on many host threads: the embarrassingly parallel upper bound SURVEY.md §8d and
    BASELINE.md:28-30 ask for beside the 1-core figure (the reference itself verifies on one
    goroutine, types/validator_set.go:685-707).  The GPU box allots one GPU's job 16 of its CPUs
    (the others belong to the jobs of the node's other GPUs), so the leg runs at 4 and 16 threads
    on the rank's NUMA node, checks that the rate scales linearly with the thread count, and
    reports the all-cores figure as the measured per-thread rate at 16 threads times the box's
    CPUs — labelled extrapolated, with the scaling it rests on beside it."""
    sys.path.insert(0, ROOT)
    from oracle import port  # cpu_baseline leg only
    box = os.cpu_count() or 1
    node = len(os.sched_getaffinity(0))
    runs = {}
    out = None
    for nt, mm in ((4, m // 4), (HOST_SHARE_THREADS, m)):
        nt = min(nt, node)
        pubs = d_pub[:mm].cpu().numpy()
        sigs = d_sig[:mm].cpu().numpy()
        o = offs[: mm + 1].astype(np.uint64)
        t = time.perf_counter()
        res = port.verify_batch(pubs, sigs, msgs, o, nthreads=nt)
        dt = time.perf_counter() - t
        runs[nt] = {"value": round(mm / dt, 1), "signatures": mm, "seconds": round(dt, 3)}
        if mm == m:
            out = res
    nt = max(runs)
    v = runs[nt]["value"]
    per_thread = v / nt
    extrap = per_thread * box
    return {"value": v, "unit": "verifies/s", "cores": nt, "kind": "port",
            "sample": "all %d signatures of the batch, %d threads, %.1f s; %s"
                      % (m, nt, runs[nt]["seconds"], _cpu_model()),
            "threads_runs": {str(k): r for k, r in sorted(runs.items())},
            "parallel_efficiency_vs_1_thread": round(per_thread / one_thread_value, 3) if one_thread_value else None,
            "box_cpus": box, "node_cpus": node, "cgroup_cpu_quota": _cgroup_cpus(),
            "all_cores_extrapolated": {
                "value": round(extrap, 1), "cores": box,
                "basis": "per-thread rate at %d threads x %d CPUs (linear: the port shares nothing between "
                         "signatures; the box allots one GPU's job %d CPUs, so %d threads are not run)"
                         % (nt, box, HOST_SHARE_THREADS, box),
                "gpu_speedup": round(gpu_value / extrap, 1) if extrap else None},
            "gpu_decisions_match": bool((d_out[:m].cpu().numpy() == out).all())}


def cpu_baseline(d_pub, d_sig, msgs, offs, m, d_out, m_ossl):
    """Single-thread C restatement of the Go verify on the first m tuples (oracle/ed25519_port.c);
    its decisions are also compared with the GPU's on that sample.  Beside it, the independent
    anchor BASELINE.md plans: OpenSSL 3 EVP_DigestVerify(ED25519), 1 thread, on the first m_ossl
    tuples of the same sample (oracle/openssl_anchor.c; absent without libcrypto)."""
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
    res = {"value": round(m / dt, 1), "unit": "verifies/s", "cores": 1, "kind": "port",
           "sample": "first %d signatures of the same batch, 1 thread, %.1f s; valid=%d; %s; host cpu_count=%d"
                     % (m, dt, int(out.sum()), _cpu_model(), ncores),
           "gpu_decisions_match": bool((gpu == out).all())}
    t = time.perf_counter()
    oo = port.openssl_verify_batch(pubs[:m_ossl], sigs[:m_ossl], msgs, o[: m_ossl + 1], nthreads=1)
    dt = time.perf_counter() - t
    if oo is not None:
        res["anchor_openssl"] = {"value": round(m_ossl / dt, 1), "unit": "verifies/s", "cores": 1,
                                 "kind": "OpenSSL 3 EVP_DigestVerify (ED25519), independent implementation",
                                 "sample": "first %d signatures of the same batch, 1 thread, %.1f s" % (m_ossl, dt),
                                 "decisions_match_port": bool((oo == out[:m_ossl]).all())}
    return res


if __name__ == "__main__":
    sys.exit(main())
