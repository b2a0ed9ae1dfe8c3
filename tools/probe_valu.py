"""Print the sustained rate of the integer VALU instructions the field code emits (tmed_valu_peak)."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tendermint-fork_amd"))
from tmed import Engine, lib  # noqa: E402

NAMES = ["v_mad_i64_i32", "v_mad_u64_u32", "v_add_u32", "v_mul_lo_u32", "v_ashrrev_i64", "v_lshl_add_u64",
         "v_lshl_add_u32", "v_add_co_u32+v_addc_co_u32", "v_lshrrev_b64", "v_alignbit_b32", "v_and_b32",
         "v_bfe_i32", "v_and_or_b32", "v_cndmask_b32 (vcc)", "v_ashrrev_i32", "v_cndmask_b32_e64 (sgpr mask)", "v_cmp+v_cndmask (vcc)", "v_cmp+v_cndmask (sgpr)"]
e = Engine(0)
l = lib()
l.tmed_valu_peak.restype = ctypes.c_int
l.tmed_valu_peak.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
res = {}
for k, name in enumerate(NAMES):
    g = ctypes.c_double(0)
    best = 0.0
    for _ in range(3):
        rc = l.tmed_valu_peak(e._h, k, ctypes.byref(g))
        assert rc == 0, rc
        best = max(best, g.value)
    res[name] = round(best / 1e3, 2)  # T lane-ops/s
full = res["v_add_u32"]
# cycles per wave instruction per SIMD at the peak engine clock (256 CUs x 4 SIMDs on MI355X)
simds, ghz = 1024, 2.4
print(json.dumps({"unit": "T lane-instructions/s", "rates": res,
                  "relative_cost_vs_add": {k: round(full / v, 2) for k, v in res.items()},
                  "cycles_per_wave_instruction_at_2.4_GHz": {k: round(simds * 64 * ghz * 1e9 / (v * 1e12), 2)
                                                             for k, v in res.items()}}, indent=1))
