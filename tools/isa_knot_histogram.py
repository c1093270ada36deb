"""Estimated per-knot instruction mix of a kernel's knot loop from a hipcc -S listing:

    python tools/isa_knot_histogram.py <listing.s> <symbol> <loop index> [inner trip count]

The loop index picks a backward-branch span (0 = the largest, the restart/knot loop); inner loops shorter than
400 instructions (the rolled `#pragma unroll 1` loops over l) are weighted by the trip count (n). A static
estimate (it counts the restart and replay paths as if taken); SQ_INSTS_VALU / waves / knots is the measured
figure to hold it against."""
import re, sys, collections
sys.path.insert(0, '/tmp/isa')
s = open(sys.argv[1]).read()
sym = sys.argv[2]
start = s.index(sym + ":"); end = s.index(".Lfunc_end", start)
body = s[start:end].split("\n")
labels = {}; ins = []
for l in body:
    m = re.match(r"^(\.LBB\S+):", l)
    if m: labels[m.group(1)] = len(ins); continue
    if l.startswith("\t") and not l.startswith("\t.") and not l.startswith("\t;") and l.strip():
        ins.append(l.strip())
loops = []
for j, l in enumerate(ins):
    m = re.match(r"s_(cbranch_\S+|branch)\s+(\.LBB\S+)", l)
    if m and m.group(2) in labels and labels[m.group(2)] <= j:
        loops.append((labels[m.group(2)], j))
loops.sort(key=lambda x: -(x[1]-x[0]))
knot = loops[int(sys.argv[3])]
inner = [lp for lp in loops if lp[0] > knot[0] and lp[1] < knot[1] and (lp[1]-lp[0]) < 400]
sel=[]
for lp in sorted(inner, key=lambda x: x[1]-x[0]):
    if not any(a<=lp[0] and lp[1]<=b for a,b in sel) and not any(lp[0]<=a and b<=lp[1] for a,b in sel): sel.append(lp)
inner=sel
print("knot loop span", knot, "inner loops", [(a,b,b-a) for a,b in inner[:12]])
w = [1.0]*len(ins)
trip = float(sys.argv[4]) if len(sys.argv) > 4 else 13.0
for a,b in inner:
    for i in range(a, b+1): w[i] *= trip
def cls(op):
    if op.startswith("v_fma_f64") or op.startswith("v_fmac_f64"): return "f64 fma"
    if op in ("v_mul_f64","v_add_f64") or op.startswith("v_mul_f64") or op.startswith("v_add_f64"): return "f64 mul/add"
    if op.startswith("v_") and "f64" in op and ("div" in op or "rcp" in op or "rsq" in op or "sqrt" in op or "ldexp" in op or "frexp" in op or "class" in op): return "f64 div/sqrt seq"
    if "dpp" in op: return "DPP move"
    if op.startswith("v_cndmask"): return "select"
    if op.startswith("v_mov"): return "v_mov"
    if op.startswith("v_cmp"): return "compare"
    if op.startswith("scratch_"): return "scratch"
    if op.startswith("ds_"): return "LDS"
    if op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_"): return "global"
    if op.startswith("v_readlane") or op.startswith("v_writelane") or op.startswith("v_readfirstlane"): return "readlane/writelane"
    if op.startswith("v_") and "f64" in op: return "f64 other"
    if op.startswith("v_"): return "int/address VALU"
    if op.startswith("s_waitcnt") or op.startswith("s_nop"): return "waitcnt/nop"
    if op.startswith("s_"): return "SALU/branch"
    return "other"
c = collections.Counter(); tot = 0.0; valu = 0.0
for i in range(knot[0], knot[1]+1):
    op = ins[i].split()[0]; k = cls(op); c[k] += w[i]; tot += w[i]
    if op.startswith("v_"): valu += w[i]
print(f"estimated dynamic instructions per knot (inner loops x {trip:g}): {tot:.0f}, VALU {valu:.0f}")
for k, v in c.most_common(): print(f"  {k:22s} {v:8.0f} {v/tot:6.1%}")
