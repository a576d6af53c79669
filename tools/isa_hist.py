"""ISA instruction histogram of a kernel's hot loop ("publish the ISA
instruction histogram per point-edge").

Extracts the gfx950 code object from a built object file (llvm-objdump --offloading), disassembles
it, finds the kernel by a substring of its mangled name, takes the largest loop (the body between a
backward branch and its target) and counts its instructions by class.  Dividing by the points the
loop body processes (the accumulate: NP points per lane and step, acc_np<MODE> in gn_accum.hip)
gives instructions per point-edge.

    python tools/isa_hist.py mast3r-slam_amd/build/gn_accum.o ILi2ELb0ELb1ELb0E 4
"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def disasm(obj):
    with tempfile.TemporaryDirectory() as d:
        tmp = os.path.join(d, os.path.basename(obj))
        subprocess.run(["cp", obj, tmp], check=True)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", tmp], check=True, cwd=d, capture_output=True)
        dev = [f for f in os.listdir(d) if "gfx950" in f]
        out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", os.path.join(d, dev[0])],
                             check=True, capture_output=True, text=True).stdout
    return out


def kernel_insns(text, key):
    lines = text.splitlines()
    start = None
    for i, l in enumerate(lines):
        m = re.match(r"^([0-9a-f]+) <(.*)>:", l)
        if m and start is not None:
            return name, base, lines[start:i]
        if m and key in m.group(2):
            start, name, base = i + 1, m.group(2), int(m.group(1), 16)
    if start is None:
        raise SystemExit(f"kernel matching {key!r} not found")
    return name, base, lines[start:]


def parse(block):
    ins, raw = [], []
    for l in block:
        m = re.match(r"^\s*(\S.*?)\s*//\s*([0-9A-Fa-f]+):", l)
        if not m:
            continue
        txt, addr = m.group(1), int(m.group(2), 16)
        ins.append((addr, txt))
        raw.append(l)
    return ins, raw


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if re.match(r"v_(sqrt|rsq|rcp|log|exp|sin|cos)_", op):
        return "valu_transcendental"
    if re.match(r"v_(fma|fmac|mac|mad|pk_fma)_", op):
        return "valu_fma"
    if re.match(r"v_(mul|pk_mul)_", op):
        return "valu_mul"
    if re.match(r"v_(add|sub|subrev|pk_add)_", op) and "_u32" not in op and "_co_" not in op and "_i32" not in op:
        return "valu_add"
    if re.match(r"v_(cndmask|cmp|cmpx)", op):
        return "valu_cmp_select"
    if re.match(r"v_(cvt|frexp|ldexp|trunc|floor|ceil|rndne|fract)", op):
        return "valu_convert"
    if re.match(r"v_(mov|readlane|readfirstlane|writelane|permlane|perm|accvgpr)", op):
        return "valu_move_permute"
    if op.startswith("v_"):
        return "valu_int_other"
    if re.match(r"(global|buffer|flat|scratch)_load", op):
        return "vmem_load"
    if re.match(r"(global|buffer|flat|scratch)_(store|atomic)", op):
        return "vmem_store"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_waitcnt"):
        return "s_waitcnt"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("s_"):
        return "salu_branch"
    return "other"


def main():
    obj, key = sys.argv[1], sys.argv[2]
    points = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
    name, base, block = kernel_insns(disasm(obj), key)
    ins, raw = parse(block)
    addrs = [a for a, _ in ins]
    loops = []
    for k, (a, t) in enumerate(ins):
        m = re.match(r"s_(cbranch_\w+|branch)\s+(\S+)", t)
        if not m:
            continue
        # llvm-objdump prints the target as <kernel+0xOFF>
        tm = re.search(r"<[^>]*\+0x([0-9a-f]+)>", raw[k])
        if not tm:
            continue
        tgt = base + int(tm.group(1), 16)
        if tgt < a and tgt in addrs:
            lo = addrs.index(tgt)
            loops.append((k - lo + 1, lo, k))
    if not loops:
        raise SystemExit("no loop found")
    # the hot loop: the longest INNERMOST loop (one that contains no other loop's back edge; the
    # outer task loop, which also holds the workgroup reduction, is excluded that way)
    inner = [(n, lo, hi) for n, lo, hi in loops
             if not any(lo <= lo2 and hi2 <= hi and (lo2, hi2) != (lo, hi) and hi2 < hi for _, lo2, hi2 in loops)]
    n, lo, hi = max(inner or loops)
    body = [t.split()[0] for _, t in ins[lo:hi + 1]]
    hist = collections.Counter(classify(op) for op in body)
    valu = sum(v for k, v in hist.items() if k.startswith("valu"))
    out = {"kernel": name, "loop_instructions": n, "points_per_iteration": points,
           "per_point_edge": {k: round(v / points, 2) for k, v in sorted(hist.items())},
           "valu_per_point_edge": round(valu / points, 2),
           "valu_f32_fma_mul_add_per_point_edge": round((hist["valu_fma"] + hist["valu_mul"] + hist["valu_add"]) / points, 2)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
