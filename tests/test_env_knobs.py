"""The product library's environment switches leave every output unchanged.

libpas.so reads a few launch-shape knobs from the environment (tuning sweeps); none of them
may change a result.  Output-changing diagnostics (ablation builds) are compile-time macros,
and the losing deschedule-kernel variants are gone, so a stray variable in a scheduler pod
cannot change filter results.
"""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "platform-aware-scheduling_amd", "lib", "libpas.so")

# output-invariant: waves per eval workgroup, segments per wave, pod order across workgroups,
# store cache policy, the global-scratch pass bitmap path, deschedule words per wave, the GAS
# fit's fork / join of its side streams (events or device flags)
INVARIANT = {"PAS_EVAL_WAVES", "PAS_EVAL_SEGS", "PAS_EVAL_NOGROUP", "PAS_EVAL_AUX",
             "PAS_EVAL_GLOBAL_PASS", "PAS_VIOL_RUN", "PAS_GAS_SYNC"}
# switches that once changed outputs (timing ablations) or picked another kernel at run time
REMOVED = {"PAS_EVAL_ABLATE": "1", "PAS_PREP_ABLATE": "3", "PAS_VIOL_FLAT": "1",
           "PAS_VIOL_DEDUP": "1", "PAS_VIOL_PAIRS": "2", "PAS_VIOL_U": "4",
           "PAS_GAS_ABLATE": "1"}


def _env_names_in_library():
    with open(LIB, "rb") as f:
        data = f.read()
    return {m.decode() for m in re.findall(rb"(?<![A-Za-z0-9_])PAS_[A-Z0-9_]+(?=\x00)", data)}


def test_library_reads_only_invariant_knobs():
    names = _env_names_in_library()
    assert names <= INVARIANT, f"unexpected environment names in libpas.so: {names - INVARIANT}"
    assert not names & set(REMOVED)


_CHILD = r"""
import sys, numpy as np
sys.path[:0] = [{root!r} + "/platform-aware-scheduling_amd", {root!r} + "/oracle"]
import oracle, pas_amd
from pas_amd import workload as wl
ctx = pas_amd.Context(0)
snap = wl.make_tas_snapshot(5000, 8, seed=0xE1)
batch = wl.make_tas_batch(snap, 24, 7, seed=0xE1, cand_frac=0.7)
ctx.tas_snapshot_set(1, snap.v_milli, snap.present)
gp, go, gl = ctx.tas_eval(1, batch.rules, batch.rule_off, batch.prio, batch.cand)
op_, oo, ol = oracle.tas_eval(snap.v_milli, snap.present, batch.rules, batch.rule_off,
                              batch.prio, batch.cand)
assert np.array_equal(gp, op_) and np.array_equal(gl, ol)
for p in range(len(gl)):
    assert np.array_equal(go[p, :gl[p]], oo[p, :ol[p]])
dr, doff = wl.make_deschedule_rules(snap, 5, 3, seed=0xE1)
assert np.array_equal(ctx.tas_violations(1, dr, doff),
                      oracle.tas_violations(snap.v_milli, snap.present, dr, doff))
gs = wl.make_gas_snapshot(1500, seed=0xE1)
gb = wl.make_gas_batch(40, seed=0xE1)
ctx.gas_snapshot_set(2, gs.n_cards, gs.cap, gs.used)
assert np.array_equal(ctx.gas_fit(2, gb.req, gb.req_mask, gb.n_containers, wl.I915),
                      oracle.gas_fit(gs.n_cards, gs.cap, gs.used, gb.req, gb.req_mask,
                                     gb.n_containers, wl.I915))
ctx.close()
print("KNOBS-OK")
"""


@pytest.mark.gpu
@pytest.mark.parametrize("knobs", [
    dict(REMOVED),
    dict(REMOVED, PAS_EVAL_WAVES="8", PAS_EVAL_SEGS="2", PAS_EVAL_NOGROUP="1", PAS_VIOL_RUN="2"),
    dict(REMOVED, PAS_EVAL_WAVES="2", PAS_EVAL_AUX="0", PAS_VIOL_RUN="16",
         PAS_EVAL_GLOBAL_PASS="1", PAS_GAS_SYNC="events"),
    dict(REMOVED, AMD_SERIALIZE_KERNEL="3"),
])
def test_env_knobs_change_no_result(knobs):
    env = dict(os.environ, **knobs)
    r = subprocess.run([sys.executable, "-c", _CHILD.format(root=ROOT)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "KNOBS-OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
