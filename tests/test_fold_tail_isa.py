"""The fused reduction tail's inter-workgroup hand-off (csrc/ssp_internal.h fold_tail), checked in the
gfx950 assembly the compiler actually emits.

The hand-off is the write-through form of /opt/skills/guides/cdna_hip_programming.md §6
Guideline 16 (R1; the split-K recipe of §5 lists it as "equally valid" to release/acquire): every
handed-off partial is stored sc1 (agent-scope relaxed atomic store) and drained with
s_waitcnt vmcnt(0) by the storing wave before the arrival counter's agent-scope atomic add, and EVERY
load of the partials in the last-arriving workgroup is an sc1 load, so the acquire is replaced by
fence(acquire, "wavefront") (compiler ordering only).  Guideline 16 asks for checks (1)-(4) in the
.s before dropping the acquire; this test performs them mechanically on every kernel that carries
the tail:
  (1) the partial stores (the last store before the first counter add) carry sc1;
  (2) an s_waitcnt vmcnt(0) lies between that store and the counter add;
  (3) the counter is an atomic (global_atomic_add);
  (4) every global load after the first counter add carries sc1 (the tail reads nothing else).
"""
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "iterative-solver_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


def kernels(text):
    name, body = None, []
    for line in text.splitlines():
        m = re.match(r"^(_Z\S+):", line)
        if m:
            name, body = m.group(1), []
            continue
        if name is not None:
            s = line.strip()
            if s and not s.startswith(";") and not s.startswith("."):
                body.append(s)
            if s.startswith("s_endpgm"):
                yield name, body
                name = None


def fold_tail_violations(ins):
    """None if the kernel has no fold tail, else the list of violated checks."""
    adds = [i for i, s in enumerate(ins) if s.startswith("global_atomic_add")]
    if not adds:
        return None
    first = adds[0]
    tail_loads = [s for s in ins[first:] if s.startswith("global_load")]
    if not any("sc1" in s for s in tail_loads):
        return None  # atomics for something else (e.g. select's compaction)
    bad = []
    stores = [i for i in range(first) if ins[i].startswith("global_store")]
    if not stores or "sc1" not in ins[stores[-1]]:
        bad.append("(1) partial store without sc1")
    elif not any(re.match(r"s_waitcnt vmcnt\(0\)", s) for s in ins[stores[-1]:first]):
        bad.append("(2) no vmcnt(0) drain before the counter add")
    bad += ["(4) tail load without sc1: " + s for s in tail_loads if "sc1" not in s]
    return bad


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_fold_tail_handoff_is_write_through_in_the_isa():
    found = 0
    with tempfile.TemporaryDirectory() as d:
        for src in ("kernels_stream.hip", "kernels_panel.hip"):
            out = os.path.join(d, src + ".s")
            r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                                "-I" + CSRC, "--cuda-device-only", "-S", os.path.join(CSRC, src), "-o", out],
                               capture_output=True, text=True, timeout=600)
            assert r.returncode == 0, r.stderr[-3000:]
            for name, ins in kernels(open(out).read()):
                bad = fold_tail_violations(ins)
                if bad is None:
                    continue
                found += 1
                assert not bad, (name, bad)
    # k_dot_partial<x==y / x!=y>, k_gemm_inner_row<1,2>, k_scal_inner / k_axpy_inner / k_axpy_norm x4
    assert found >= 16, found
