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
  (1) the partial stores (the nearest store before the first counter add) carry sc1;
  (2) an s_waitcnt vmcnt(0) lies between that store and the counter add;
  (3) the counter is an atomic (global_atomic_add);
  (4) every global load after the first counter add carries sc1 (the tail reads nothing else).
"Before" and "after" follow the kernel's control-flow graph, not the order of the text: the compiler
lays blocks out after an s_endpgm (early returns, loop remainders).
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
            if s.startswith(".Lfunc_end"):  # a kernel may hold several s_endpgm (early returns)
                yield name, body
                name = None
            elif s and not s.startswith(";") and (not s.startswith(".") or re.match(r"^\.LBB\S*:", s)):
                body.append(s.split(";")[0].strip())


def cfg(ins):
    """Basic blocks of a kernel body: (starts, succ, pred, block_of) over instruction indices.  Labels
    (".LBB..:") are kept in `ins` by kernels(); the compiler may lay blocks out after an s_endpgm (loop
    remainders, early exits), so the order of the text is not the order of execution."""
    label_at = {s[:-1]: i for i, s in enumerate(ins) if re.match(r"^\.LBB\S*:$", s)}
    starts = sorted({0} | set(label_at.values())
                    | {i + 1 for i, s in enumerate(ins) if re.match(r"s_(c?branch|endpgm)", s) and i + 1 < len(ins)})
    block_of = {}
    for b, st in enumerate(starts):
        for i in range(st, starts[b + 1] if b + 1 < len(starts) else len(ins)):
            block_of[i] = b
    succ = {b: set() for b in range(len(starts))}
    for b, st in enumerate(starts):
        end = (starts[b + 1] if b + 1 < len(starts) else len(ins)) - 1
        last = ins[end]
        m = re.match(r"s_(c?branch)\S*\s+(\.LBB\S+)", last)
        if m:
            succ[b].add(block_of[label_at[m.group(2)]])
        if not (last.startswith("s_endpgm") or last.startswith("s_branch ")) and b + 1 < len(starts):
            succ[b].add(b + 1)
    pred = {b: set() for b in succ}
    for b, ss in succ.items():
        for s in ss:
            pred[s].add(b)
    return starts, succ, pred, block_of


def fold_tail_violations(ins):
    """None if the kernel has no fold tail, else the list of violated checks."""
    adds = [i for i, s in enumerate(ins) if s.startswith("global_atomic_add")]
    if not adds:
        return None
    first = adds[0]
    starts, succ, pred, block_of = cfg(ins)
    bounds = lambda b: (starts[b], starts[b + 1] if b + 1 < len(starts) else len(ins))
    # the tail: everything reachable from the first counter add
    tail_loads, seen, work = [], set(), [block_of[first]]
    while work:
        b = work.pop()
        if b in seen:
            continue
        seen.add(b)
        lo, hi = bounds(b)
        tail_loads += [ins[i] for i in range(first + 1 if b == block_of[first] else lo, hi)
                       if ins[i].startswith("global_load")]
        work += succ[b]
    if any(block_of[first] in succ[b] for b in seen):  # the add's own block is re-entered (a loop)
        lo, _ = bounds(block_of[first])
        tail_loads += [ins[i] for i in range(lo, first) if ins[i].startswith("global_load")]
    if not any("sc1" in s for s in tail_loads):
        return None  # atomics for something else (e.g. select's compaction)
    bad = []
    # (1)/(2): walk backwards from the add along every path to the nearest global store.  A path whose
    # lanes store no partial (an execz skip round the store) reaches an earlier streaming store instead,
    # so (1) asks that the partial store -- an sc1 store -- is nearest on some path, and (2) that every
    # path drains with vmcnt(0) whatever store it meets.
    nearest, seen, work = [], set(), [(block_of[first], first - 1, False)]
    while work:
        b, i, drained = work.pop()
        lo, _ = bounds(b)
        while i >= lo and not ins[i].startswith("global_store"):
            drained |= bool(re.match(r"s_waitcnt vmcnt\(0\)", ins[i]))
            i -= 1
        if i >= lo:
            nearest.append(ins[i])
            if not drained:
                bad.append("(2) no vmcnt(0) drain between " + ins[i] + " and the counter add")
            continue
        for p in pred[b]:
            if (p, drained) not in seen:
                seen.add((p, drained))
                work.append((p, bounds(p)[1] - 1, drained))
    if not any("sc1" in s for s in nearest):
        bad.append("(1) partial store without sc1: " + str(nearest))
    bad += ["(4) tail load without sc1: " + s for s in tail_loads if "sc1" not in s]
    return bad


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_fold_tail_handoff_is_write_through_in_the_isa():
    found, names = 0, []
    with tempfile.TemporaryDirectory() as d:
        for src in ("kernels_stream.hip", "kernels_panel.hip", "kernels_exact.hip", "kernels_sparse.hip"):
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
                names.append(name)
                assert not bad, (name, bad)
    # k_dot_partial<x==y / x!=y>, k_gemm_inner_row<1,2>, k_scal_inner / k_axpy_inner / k_axpy_norm x4,
    # and the publish tails of the short-vector dot (kernels_exact.hip) and the inline sparse inner
    # products (kernels_sparse.hip)
    assert found >= 18, found
    for kernel in ("k_exact_inner", "k_sparse_inner_inline"):
        assert any(kernel in nm for nm in names), (kernel, names)



GOOD = """
_Zk:
  global_load_dwordx2 v[0:1], v2, s[0:1]
  global_store_dwordx2 v2, v[0:1], s[0:1] sc1
  s_cbranch_execz .LBB0_2
  s_waitcnt vmcnt(0)
  global_atomic_add v3, v2, v3, s[2:3] sc0
  global_load_dwordx2 v[8:9], v6, s[0:1] sc1
  s_cbranch_scc1 .LBB0_3
.LBB0_1:
  s_endpgm
.LBB0_2:
  s_branch .LBB0_1
.LBB0_3:
  global_load_dwordx2 v[4:5], v6, s[0:1] offset:8 sc1
  s_branch .LBB0_1
.Lfunc_end0:
"""


def test_the_checker_follows_the_control_flow_not_the_layout():
    def check(text):
        (_, ins), = kernels(text)
        return fold_tail_violations(ins)
    assert check(GOOD) == []
    # a tail load laid out after the s_endpgm, reached through the branch after the add
    assert [v[:3] for v in check(GOOD.replace("offset:8 sc1", "offset:8"))] == ["(4)"]
    assert [v[:3] for v in check(GOOD.replace("  s_waitcnt vmcnt(0)\n", ""))] == ["(2)"]
    assert [v[:3] for v in check(GOOD.replace("s[0:1] sc1\n  s_cbranch_execz", "s[0:1]\n  s_cbranch_execz"))] == ["(1)"]


def store_drain_violations(ins):
    """(1)-(3) without (4), for a publishing pass whose last arriver reads nothing back: the nearest
    store before the first counter add carries sc1 on some path and every path drains vmcnt(0)."""
    adds = [i for i, s in enumerate(ins) if s.startswith("global_atomic_add")]
    if not adds:
        return ["(3) no counter add"]
    first = adds[0]
    starts, succ, pred, block_of = cfg(ins)
    bounds = lambda b: (starts[b], starts[b + 1] if b + 1 < len(starts) else len(ins))
    bad, nearest, seen, work = [], [], set(), [(block_of[first], first - 1, False)]
    while work:
        b, i, drained = work.pop()
        lo, _ = bounds(b)
        while i >= lo and not ins[i].startswith("global_store"):
            drained |= bool(re.match(r"s_waitcnt vmcnt\(0\)", ins[i]))
            i -= 1
        if i >= lo:
            nearest.append(ins[i])
            if not drained:
                bad.append("(2) no vmcnt(0) drain between " + ins[i] + " and the counter add")
            continue
        for p in pred[b]:
            if (p, drained) not in seen:
                seen.add((p, drained))
                work.append((p, bounds(p)[1] - 1, drained))
    if not any("sc1" in s for s in nearest):
        bad.append("(1) published store without sc1: " + str(nearest))
    return bad


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_reduce_pass_publishes_before_it_arrives():
    """k_reduce_publish (the gemm_inner panels' reduce pass with one rank): each workgroup's sum is a
    system-scope (sc0 sc1) store drained with vmcnt(0) before the arrival counter's atomic add, so the
    last arriver's flag follows every sum into host memory."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "kernels_stream.s")
        r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                            "-I" + CSRC, "--cuda-device-only", "-S", os.path.join(CSRC, "kernels_stream.hip"), "-o", out],
                           capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
        found = [(name, store_drain_violations(ins)) for name, ins in kernels(open(out).read())
                 if "k_reduce_publish" in name]
    assert found, "k_reduce_publish not emitted"
    for name, bad in found:
        assert not bad, (name, bad)


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_select_lists_reach_the_last_workgroup_write_through():
    """k_select_local: each workgroup's list is stored write-through (sc1) and drained before the
    arrival add, and the last arriver reads the lists with sc1 loads.  Its only other loads after the
    add are of the input shard (the selected elements' returned values: x, and y for select_max_dot),
    which no workgroup of the launch writes."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "kernels_select.s")
        r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                            "-I" + CSRC, "--cuda-device-only", "-S", os.path.join(CSRC, "kernels_select.hip"), "-o", out],
                           capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
        found = [(name, fold_tail_violations(ins)) for name, ins in kernels(open(out).read())
                 if "k_select_local" in name]
    assert len(found) == 4, [n for n, _ in found]
    for name, bad in found:
        assert bad is not None, name
        inputs = 2 if "k_select_localILi1E" in name else 1
        assert all(b.startswith("(4) tail load without sc1") for b in bad), (name, bad)
        assert len(bad) <= inputs, (name, bad)
