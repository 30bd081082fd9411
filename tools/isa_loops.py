"""Loop census of a hipcc -S (or --save-temps) gfx950 assembly file.

  python tools/isa_loops.py <file.s> <kernel-name-substring> [--dump]

For every backward branch of the matching kernel prints the loop body's size and counts per
instruction class (MFMA, ds_read, ds_write, LDS-DMA buffer loads, other VMEM, accvgpr moves,
VALU, SALU, waitcnts, barriers) — the quick check that a main loop is what the source intends
(no accumulator copies through the loop phis, no vmcnt(0) in the steady state, no scratch).
"""
import re
import sys
from collections import Counter


def classify(ins):
    op = ins.split()[0]
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_accvgpr_read"):
        return "accvgpr_read"
    if op.startswith("v_accvgpr_write"):
        return "accvgpr_write"
    if op.startswith("v_accvgpr_mov"):
        return "accvgpr_mov"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "ds_read"
    if op.startswith("ds_write") or op.startswith("ds_store"):
        return "ds_write"
    if op.startswith("ds_"):
        return "ds_other"
    if (op.startswith("buffer_load") or op.startswith("global_load")) and " lds" in ins:
        return "vmem_lds"
    if op.startswith(("buffer_load", "global_load", "flat_load")):
        return "vmem_load"
    if op.startswith(("buffer_store", "global_store", "flat_store")):
        return "vmem_store"
    if op.startswith("scratch_"):
        return "SCRATCH"
    if op == "s_waitcnt":
        return "waitcnt"
    if op == "s_barrier":
        return "barrier"
    if op.startswith("s_nop"):
        return "s_nop"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    dump = "--dump" in sys.argv
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if re.match(r"^[\w.$]+:", l) and name in l.split(":")[0] and not l.startswith("."):
            start = i
            break
    if start is None:
        sys.exit(f"kernel {name} not found")
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    print(lines[start].split(":")[0])
    labels = {}
    for k, l in enumerate(body):
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            labels[m.group(1)] = k
    insts = [(k, l.strip()) for k, l in enumerate(body)
             if l.startswith("\t") and not l.strip().startswith((";", ".")) and l.strip()]
    total = Counter(classify(t) for _, t in insts)
    print("whole kernel:", dict(total))
    for k, l in enumerate(body):
        m = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
        if not m:
            continue
        tk = labels[m.group(1)]
        if tk >= k:
            continue
        loop = [t for kk, t in insts if tk <= kk <= k]
        c = Counter(classify(t) for t in loop)
        waits = Counter(t for t in loop if t.startswith("s_waitcnt"))
        print(f"\nloop {m.group(1)} lines {tk}-{k}: {len(loop)} instructions")
        print("  ", dict(sorted(c.items(), key=lambda x: -x[1])))
        print("   waitcnts:", dict(waits))
        if dump:
            for t in loop:
                print("     ", t)


if __name__ == "__main__":
    main()
