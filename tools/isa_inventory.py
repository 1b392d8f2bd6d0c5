"""ISA inventory of a kernel loop: instruction classes per basic block and in total.

python tools/isa_inventory.py <file.s> <function-symbol-substring> <loop-header-label>

Reads hipcc --save-temps assembly, takes the function whose symbol contains the given substring,
and the blocks annotated "in Loop: Header=<label>" (plus the header), and counts VALU instructions
by class: binary64 arithmetic, 64-bit address arithmetic, v_cndmask / moves, compares, integer /
bit ops, f32, other; plus SALU, branches, memory and waitcnt.  Static counts (each instruction
once); DESIGN.md §5.15 weighs them with the blocks' execution frequencies where it matters."""
import re
import sys
from collections import Counter, OrderedDict


def classify(op):
    if op.startswith("s_waitcnt") or op.startswith("s_nop"):
        return "wait/nop"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("global_", "flat_", "buffer_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if not op.startswith("v_"):
        return "other"
    if op.startswith("v_cmp") or op.startswith("v_cmpx"):
        return "valu cmp"
    if op.startswith("v_cndmask"):
        return "valu cndmask"
    if op.startswith(("v_mov", "v_readlane", "v_writelane", "v_readfirstlane", "v_accvgpr")):
        return "valu mov/lane"
    if "f64" in op or op.startswith("v_div_f") and "f64" in op:
        return "valu f64"
    if op in ("v_lshl_add_u64", "v_lshlrev_b64", "v_mad_u64_u32", "v_add_co_u32_e32", "v_addc_co_u32_e32",
              "v_add_co_u32_e64", "v_addc_co_u32_e64", "v_ashrrev_i64", "v_lshrrev_b64", "v_mad_i64_i32"):
        return "valu addr64"
    if "f32" in op or "f16" in op:
        return "valu f32"
    return "valu int/bit"


def main():
    path, fsub, header = sys.argv[1], sys.argv[2], sys.argv[3]
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^\S*%s\S*:" % re.escape(fsub), l))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    blocks = OrderedDict()
    tag = "Header=" + header.lstrip(".").lstrip("L")          # .LBB6_509 -> Header=BB6_509
    cur = None
    for l in lines[start:end]:
        m = re.match(r"^(\.LBB\S+|; %bb\.\d+):", l)
        if m:
            cur = m.group(1).lstrip("; %")
            blocks[cur] = [cur == header, Counter()]
        if cur is None:
            continue
        if tag in l:
            blocks[cur][0] = True
        s = l.split(";")[0].strip()
        if not s or s.endswith(":") or s.startswith("."):
            continue
        blocks[cur][1][classify(s.split()[0])] += 1
    tot = Counter()
    nb = 0
    for name, (inl, c) in blocks.items():
        if inl:
            tot.update(c)
            nb += 1
    valu = sum(v for k, v in tot.items() if k.startswith("valu"))
    print("loop %s of %s: %d blocks, %d instructions, %d VALU" % (header, fsub, nb, sum(tot.values()), valu))
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print("  %-14s %5d  %5.1f%% of VALU" % (k, v, 100.0 * v / valu if k.startswith("valu") else float("nan")))


if __name__ == "__main__":
    main()
