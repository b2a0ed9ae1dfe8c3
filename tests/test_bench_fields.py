"""bench.py's reporting logic, CPU only (the GPU legs themselves run on the box): the compact `legs`
summary that ends every line (so the driver's stdout tail carries every leg), and the archived PMC
fields, reported only when profiles/pmc_summary.json was collected on this tree's kernel sources."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tendermint-fork_amd")]

import bench  # noqa: E402


def _result():
    return {"value": 108.1e6, "ms_per_step": 9.697, "roofline": {"frac": 0.5723, "prep_kernels_ms": 2.2112},
            "c2_keyset_variant": {"value": 578e6, "ms_per_step": 1.813, "roofline": {"frac": 0.57}},
            "c1_verifycommit_p50": {"paths": {"cache_hit": {"p50_ms": 0.0794},
                                              "first_call_after_set_change": {"p50_ms": 0.2476},
                                              "first_call_after_warmed_set_change": {"p50_ms": 0.0849},
                                              "generic_cache_off": {"p50_ms": 0.2347}},
                                    "cpu_baseline": {"value": 6.608}},
            "c3_light_client": {"direct": {"headers_per_s": 1.45e6, "headers_per_s_incl_marshal": 0.89e6,
                                           "phase_share": {"plan_frac": 0.583}, "outcome_mismatches": 0},
                                "bisection": {"headers_per_s": 264403.4}},
            "c4_shard": {"value": 592e6, "value_incl_marshal": 406e6, "value_incl_marshal_overlapped": 553e6,
                         "outcome_mismatches": 0},
            "c5": {"value": 106e6, "mismatches_vs_port": 0},
            "zip215_batch_mode": {"c2": {"value": 178e6, "mismatches_vs_port_zip215": 0},
                                  "c5": {"value": 104e6, "mismatches_vs_port_zip215": 0}},
            "cpu_baseline": {"value": 26920.4, "gpu_speedup_vs_1_core": 4015.6,
                             "all_cores": {"measured_threads": 16, "measured_value": 418105.8,
                                           "extrapolated_cores": 256, "extrapolated_value": 6.69e6,
                                           "gpu_speedup_vs_all_cores": 16.2}}}


def test_legs_summary_is_short_and_complete():
    legs = bench.legs_summary(_result())
    s = json.dumps(legs)
    assert len(s) < 1000, len(s)  # well inside the driver's 2,000-character stdout tail
    assert legs["c2_Mps"] == 108.1 and legs["prep_ms"] == 2.2112
    assert legs["c2_keyed"]["Mps"] == 578.0
    assert legs["c1_ms"]["hit"] == 0.0794 and legs["c1_ms"]["cpu"] == 6.608
    assert legs["c3"]["plan_frac"] == 0.583 and legs["c3"]["mismatches"] == 0
    assert legs["c4"]["overlapped_Mps"] == 553.0
    assert legs["c5"]["mismatches"] == 0 and legs["zip215"]["mismatches"] == 0
    assert legs["cpu"]["all_cores"] == 256 and legs["cpu"]["x_all"] == 16.2


def test_legs_summary_tolerates_skipped_legs():
    r = {"value": 1e8, "ms_per_step": 10.0, "roofline": None, "c5": None, "cpu_baseline": None}
    legs = bench.legs_summary(r)
    assert legs["c2_Mps"] == 100.0 and "c5" not in legs and "cpu" not in legs


def test_archived_pmc_only_for_this_trees_kernels(tmp_path, monkeypatch):
    """A summary tagged with another kernel-source digest is not reported (traffic None, with the
    reason); with the matching digest its fields come back."""
    from tmed.srcdigest import kernel_src_digest
    prof = tmp_path / "profiles"
    prof.mkdir()
    summ = {"verify_main_hs_kernel": {"hbm_bytes_per_sig": 100.0, "effective_clock_ghz": 2.0},
            "_meta": {"kernel_src_sha16": "0000000000000000"}}
    (prof / "pmc_summary.json").write_text(json.dumps(summ))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    t, why = bench.pmc_traffic(1 << 20)
    assert t is None and "kernel sources" in why
    assert bench.pmc_clock("verify_main_hs_kernel") is None
    summ["_meta"]["kernel_src_sha16"] = kernel_src_digest()
    (prof / "pmc_summary.json").write_text(json.dumps(summ))
    t, src = bench.pmc_traffic(1 << 20)
    assert t == 100 * (1 << 20) and "verify_main_hs_kernel" in src
    assert bench.pmc_clock("verify_main_hs_kernel") == 2.0


def test_kernel_digest_tracks_device_sources(tmp_path):
    """The digest covers kernels.hip and every csrc header, nothing else."""
    from tmed.srcdigest import kernel_src_digest
    for f in ("kernels.hip", "a.h", "b.h"):
        (tmp_path / f).write_text(f)
    d0 = kernel_src_digest(str(tmp_path))
    (tmp_path / "commit.hip").write_text("host only")
    assert kernel_src_digest(str(tmp_path)) == d0
    (tmp_path / "b.h").write_text("changed")
    assert kernel_src_digest(str(tmp_path)) != d0
