"""Instruction statistics of a kernel (and the device functions it calls) in a hipcc -S listing.

  python tools/isa_stats.py <file.s> <symbol-regex>
Prints, per matching symbol: instruction count, scalar loads, waitcnts, scratch ops, fp64 VALU ops, calls,
and the VGPR/AGPR/scratch figures from the listing's metadata."""
import re
import sys
from collections import Counter


def functions(s):
    for m in re.finditer(r"^(\S+):\s*;\s*@(\S+)\n", s, re.M):
        start = m.end()
        end = s.find(".Lfunc_end", start)
        yield m.group(1), s[start:end], end


def stats(body):
    ops = Counter()
    for l in body.split("\n"):
        if l.startswith("\t") and not l.startswith("\t.") and not l.startswith("\t;"):
            ops[l.split()[0]] += 1
    return ops


def main():
    s = open(sys.argv[1]).read()
    pat = re.compile(sys.argv[2])
    for name, body, end in functions(s):
        if not pat.search(name):
            continue
        ops = stats(body)
        tail = s[end:end + 4000]
        meta = {k: re.search(r";\s*" + k + r":\s*(\S+)", tail) for k in ("NumVgprs", "NumAgprs", "ScratchSize", "Occupancy")}
        meta = {k: (v.group(1) if v else "?") for k, v in meta.items()}
        calls = re.findall(r"s_(?:swappc|getpc)_b64.*|\ts_add_u32\s+s\d+, s\d+, (\S+)@rel32@lo", body)
        callees = sorted(set(re.findall(r"(\S+)@rel32@lo", body)))
        tot = sum(ops.values())
        f64 = sum(v for k, v in ops.items() if k.startswith("v_") and "f64" in k)
        sl = sum(v for k, v in ops.items() if k.startswith("s_load") or k.startswith("s_buffer_load"))
        scr = sum(v for k, v in ops.items() if k.startswith("scratch_") or k.startswith("buffer_"))
        print(f"{name[:100]}\n  instr {tot} f64 {f64} s_load {sl} waitcnt {ops['s_waitcnt']} scratch {scr} "
              f"calls {ops['s_swappc_b64']} {meta}")
        for c in callees:
            print("   calls", c[:100])
        top = ", ".join(f"{k} {v}" for k, v in ops.most_common(14))
        print("  top:", top)


if __name__ == "__main__":
    main()
