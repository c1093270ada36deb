"""Build ab_var/prof_inf/libtog.so: the main build's objects with k_inf_quadrotor.o recompiled from a
patched copy of tog_kernels.hpp that carries BPROF section timers in k_backward (-DTOG_BWD_PROF), and
tog_bwd_prof_read in that translation unit. The repository's sources are not modified (the copy lives in
/tmp). Run here after the main build; then on the GPU box: TOG_LIBRARY=ab_var/prof_inf/libtog.so
python tools/bwd_prof_inf.py."""
import os
import pathlib
import re
import shutil
import subprocess

ROOT = pathlib.Path(__file__).resolve().parents[1]
PKG = next(p for p in ROOT.iterdir() if p.name.endswith("_amd"))
CS = PKG / "csrc"
TMP = pathlib.Path("/tmp/vprof")
shutil.rmtree(TMP, ignore_errors=True)
(TMP / "pkg" / "csrc").mkdir(parents=True)
shutil.copytree(ROOT / "include", TMP / "include")
for f in CS.glob("*.hpp"):
    shutil.copy(f, TMP / "pkg" / "csrc" / f.name)
src = (CS / "tog_kernels.hpp").read_text()
i0 = src.index("__global__ void __launch_bounds__(64) k_backward(")
i1 = src.index("// k_forward: forwardpass!")
kb = src[i0:i1]
rep = [
    ("attempt:\n", "BPROF_DECL\nattempt:\n"),
    ("  for (int k = N - 2; k >= 0; k--) {\n", "  for (int k = N - 2; k >= 0; k--) {\n    BPROF(5);\n"),
    ("    else if (lane < n + m) sh.uk[lane - n] = Ug[(size_t)k * m + lane - n];\n    wsync();\n",
     "    else if (lane < n + m) sh.uk[lane - n] = Ug[(size_t)k * m + lane - n];\n    wsync();\n    BPROF(0);\n"),
    ("      bwd_expand<M, SQRT, AL>(P, Bf, b, k, sh);\n    }\n    wsync();\n",
     "      bwd_expand<M, SQRT, AL>(P, Bf, b, k, sh);\n    }\n    wsync();\n    BPROF(1);\n"),
    ("    if (faithful) {\n      bwd_store_q", "    BPROF(2);\n    if (faithful) {\n      bwd_store_q"),
    ("    // ---- gains: K = -(Quu_reg", "    BPROF(3);\n    // ---- gains: K = -(Quu_reg"),
    ("    // ---- write K[k], d[k]", "    BPROF(4);\n    // ---- write K[k], d[k]"),
    ("  if (!aborted) reg_decrease(P, s);", "  BPROF(6);\n  BPROF_FLUSH\n  if (!aborted) reg_decrease(P, s);"),
]
for a, b in rep:
    assert kb.count(a) == 1, a
    kb = kb.replace(a, b)
rest = src[i1:]
j0 = rest.index("// Section timers of the knot loop")
j1 = rest.index("#define BPROF_FLUSH\n#endif\n", j0) + len("#define BPROF_FLUSH\n#endif\n")
timers = rest[j0:j1]
rest = rest[:j0] + rest[j1:]
head = src[:i0]
t0 = head.rindex("template <class M, int SQRTI, int ALI>")  # the line before k_backward's signature
(TMP / "pkg" / "csrc" / "tog_kernels.hpp").write_text(head[:t0] + timers + head[t0:] + kb + rest)
tu = (CS / "k_inf_quadrotor.hip").read_text() + '''
extern "C" int tog_bwd_prof_read(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(tog::tog_bwd_prof), sizeof(unsigned long long) * tog::BPROF_N) != hipSuccess)
    return -1;
  unsigned long long z[tog::BPROF_N] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(tog::tog_bwd_prof), z, sizeof(z)) == hipSuccess ? tog::BPROF_N : -1;
}
'''
(TMP / "pkg" / "csrc" / "k_inf_quadrotor.hip").write_text(tu)
mk = (CS / "Makefile").read_text()
hdrs = re.search(r"^HDRS = (.*)$", mk, re.M).group(1).split()
h = subprocess.run("cat " + " ".join(hdrs) + " | sha1sum", shell=True, cwd=CS, capture_output=True, text=True,
                   check=True).stdout[:15]
flags = ["-O3", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950", "-fPIC", "-Wall", "-Wno-unused-function",
         f"-DTOG_HEADER_HASH=0x{h}LL", "-DTOG_BWD_PROF"]
subprocess.run(["/opt/rocm/bin/hipcc", *flags, "-c", "k_inf_quadrotor.hip", "-o", "k_inf_quadrotor.o"],
               cwd=TMP / "pkg" / "csrc", check=True)
objs = [str(CS / o) for o in ["tog_runtime.o", "tog_altro.o", "k_quadrotor_jac.o"]]
models = re.search(r"^MODELS = (.*)$", mk, re.M).group(1).split()
for mname in models:
    objs.append(str(TMP / "pkg" / "csrc" / "k_inf_quadrotor.o") if mname == "inf_quadrotor" else str(CS / f"k_{mname}.o"))
out = ROOT / "ab_var" / "prof_inf"
out.mkdir(parents=True, exist_ok=True)
subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "--offload-arch=gfx950", "-fPIC", "-o", str(out / "libtog.so"), *objs],
               check=True)
print("built", out / "libtog.so")
