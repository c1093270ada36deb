#!/usr/bin/env python3
"""Static instruction mix of one kernel in a hipcc -save-temps .s file, per source line.

usage: isa_stats.py <file.s> <kernel-substring> [source-file-substring] [top]
Counts instructions by class (VALU, DPP, LDS, SMEM, VMEM, scratch, SALU, branch) per `.loc`
source line of the given header, so the heaviest lines of the unrolled code stand out.
"""
import collections
import re
import sys


def klass(op: str, line: str) -> str:
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        if "dpp" in line or "row_" in line:
            return "dpp"
        if "_f64" in op or op.startswith(("v_fma_f64", "v_mul_f64", "v_add_f64")):
            return "valu64"
        return "valu"
    return "other"


def main():
    path, pat = sys.argv[1], sys.argv[2]
    src = sys.argv[3] if len(sys.argv) > 3 else "tog_bwd_team.hpp"
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 40
    lines = open(path).read().split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and pat in l]
    files = {}
    for l in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2))
    for a in starts:
        b = a + 1
        while not lines[b].startswith(".Lfunc_end"):
            b += 1
        per = collections.defaultdict(collections.Counter)
        tot = collections.Counter()
        ops = collections.Counter()
        cur = None
        for l in lines[a:b]:
            t = l.strip()
            if t.startswith(".loc"):
                f = t.split()[1]
                ln = int(t.split()[2])
                cur = (files.get(f, f).split("/")[-1], ln)
                continue
            if not t or t.startswith((".", ";")) or t.endswith(":"):
                continue
            op = t.split()[0]
            k = klass(op, t)
            tot[k] += 1
            ops[op] += 1
            key = cur if cur and src in cur[0] else ("other", 0)
            per[key][k] += 1
        print(lines[a].split(":")[0][:90])
        print("  total", sum(tot.values()), dict(tot.most_common()))
        print("  top ops", ops.most_common(25))
        rank = sorted(per.items(), key=lambda kv: -sum(v for k, v in kv[1].items() if k in ("valu", "valu64", "dpp")))
        for key, c in rank[:top]:
            print(f"  {key[0]}:{key[1]:5d}  " + " ".join(f"{k}={v}" for k, v in c.most_common()))


if __name__ == "__main__":
    main()
