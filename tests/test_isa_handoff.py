"""CPU: the row fill's counted waits, checked on the shipped gfx950 ISA.

nw_fill_rows_kernel (the configs[0]/[3] column-stripe fill) prefetches the
next 8-row group of its left neighbour's boundary column with an inline-asm
`global_load_dwordx2 ... sc1` and waits for it one group later with a
hand-counted `s_waitcnt vmcnt(N)` (nw_kernels.hip, `rows`): N = the VMEM
operations the group issues after the prefetch (8 mask + 8 boundary stores,
score-only 8 boundary stores).  The compiler does not see that load, so this
test walks every path of the disassembled code object from each such load to
the wait that retires it (tools/isa_check.py) and asserts, for every
instantiation (K = 1, 2 x walk / full / no codes x both penalty forms x
the three placements):

* exactly N VMEM operations are issued between the prefetch and its wait on
  every path (fewer: the wait returns before the data lands; more: a slower
  wait than the source claims);
* no instruction on those paths touches the load's destination VGPRs (a
  read sees stale data; a write is overwritten when the load lands - the
  round-2 clamped-prefetch failure);
* no path reaches s_endpgm with the load in flight (the last group issues
  no prefetch).

Reference path: the fill loop, needleman_wunsch_affine.rs:217-236.
"""
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

OBJ = os.path.join(ROOT, "sequencealigning_amd", "build", "nw_kernels.o")
LIB = os.path.join(ROOT, "sequencealigning_amd", "libsaln.so")


@pytest.fixture(scope="module")
def rows_kernels():
    import isa_check
    if not os.path.exists(OBJ):
        pytest.fail(f"{OBJ} missing: run __graft_entry__.build() first")
    if os.path.exists(LIB):
        assert os.path.getmtime(OBJ) <= os.path.getmtime(LIB) + 1, \
            "build/nw_kernels.o is newer than libsaln.so: rebuild"
    funcs = isa_check.load_functions(OBJ)
    out = {}
    for name, insns in funcs.items():
        m = re.search(r"nw_fill_rows_kernelILi(\d)ELi(\d)ELb(\d)ELi(\d)E", name)
        if m:
            out[tuple(int(m.group(i)) for i in range(1, 5))] = insns
    return out


# (K, codes, minpen, placement): every instantiation (placement 2, XCD-local
# neighbours, holds a plain-publication and an sc1-publication body)
KEYS = [(k, c, p, pl) for k in (1, 2) for c in (0, 1, 2) for p in (0, 1) for pl in (0, 1, 2)]


def test_all_row_fill_instantiations_present(rows_kernels):
    assert set(rows_kernels) == set(KEYS)


@pytest.mark.parametrize("key", KEYS, ids=lambda k: f"K{k[0]}_codes{k[1]}_minpen{k[2]}_place{k[3]}")
def test_prefetch_counted_wait_exact(rows_kernels, key):
    import isa_check
    insns = rows_kernels[key]
    expect = 8 if key[1] == 2 else 16  # kCodesNone: boundary stores only
    reps = isa_check.check_function(
        insns, pick=lambda i: i.op == "global_load_dwordx2" and i.args.rstrip().endswith("sc1"))
    assert reps, "no sc1 boundary loads found"
    counted = []
    for r in reps:
        where = f"{r.insn.addr:#x} {r.insn.op} {r.insn.args}"
        assert not r.clobbers, f"{where}: destination touched before its wait: {sorted(r.clobbers)[:3]}"
        assert not r.unwaited_exit, f"{where}: in flight at s_endpgm"
        assert r.waits, f"{where}: no wait retires it"
        for addr, n, cnt in r.waits:
            assert cnt == n, f"{where}: wait {addr:#x} vmcnt({n}) after {cnt} VMEM ops"
            if n:
                counted.append(n)
    # the group prefetch (the poll loop's and the first group's loads wait vmcnt(0))
    assert counted and set(counted) == {expect}


@pytest.mark.parametrize("key", KEYS, ids=lambda k: f"K{k[0]}_codes{k[1]}_minpen{k[2]}_place{k[3]}")
def test_publication_forms(rows_kernels, key):
    """The visibility rule of the boundary hand-off (DESIGN.md §3 "Hand-off
    rules", MI355X_MICROARCH.md "Workgroup dispatch, XCD placement &
    inter-workgroup visibility"), on the shipped ISA:

    * every boundary load is a vector `global_load_dwordx2 ... sc1` (L1
      bypassed, L2-served: never a stale L1 line, never a scalar load);
    * the dispatch-order placements (0, 1) publish every row with
      `global_store_dwordx2 ... sc1` (write-through: visible from any XCD);
    * the XCD-run placement (2) also holds the plain form (the line stays in
      the producer's L2, which its same-XCD consumer's sc1 load reads) and
      the co-location check that selects it: one `global_store_dword ... sc1`
      posting the wave's {epoch, XCC_ID} slot and `global_load_dword ... sc1`
      polls of the consumer's slot, vector forms only."""
    insns = rows_kernels[key]
    sc1 = lambda i: i.args.rstrip().endswith("sc1")  # noqa: E731
    x2_loads = [i for i in insns if i.op == "global_load_dwordx2"]
    assert x2_loads and all(sc1(i) for i in x2_loads)
    assert not any(i.op.startswith("flat_load") for i in insns)
    pub = [i for i in insns if i.op == "global_store_dwordx2"]
    plain = [i for i in pub if not sc1(i)]
    slot_posts = [i for i in insns if i.op == "global_store_dword" and sc1(i)]
    slot_polls = [i for i in insns if i.op == "global_load_dword" and sc1(i)]
    assert any(sc1(i) for i in pub)
    if key[3] == 2:
        assert plain and len(slot_posts) == 1 and slot_polls
        assert slot_posts[0].addr < min(i.addr for i in slot_polls)
    else:
        assert not plain and not slot_posts and not slot_polls
