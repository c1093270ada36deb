"""Build ab_var/kuka_helper/libtog.so: the main build's objects with k_mt_kuka.o recompiled with
-DTOG_KUKA_HELPER_F, i.e. Kuka::f written through the chol()/solve() helpers (round 4's form, whose
MinTime<Kuka> rollouts accepted diverged trials, profiles/r4j_mt_kuka_trials_split_f.txt). For the
investigation only: run the regression test against it on the GPU box with
TOG_LIBRARY=ab_var/kuka_helper/libtog.so, and compare the two forms' ISA (--isa: both listings of
k_mt_kuka.hip into /tmp/kuka_isa/). Run here after the main build."""
import pathlib
import re
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
PKG = next(p for p in ROOT.iterdir() if p.name.endswith("_amd"))
CS = PKG / "csrc"
mk = (CS / "Makefile").read_text()
hdrs = re.search(r"^HDRS = (.*)$", mk, re.M).group(1).split()
h = subprocess.run("cat " + " ".join(hdrs) + " | sha1sum", shell=True, cwd=CS, capture_output=True, text=True,
                   check=True).stdout[:15]
flags = ["-O3", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950", "-fPIC", "-Wall", "-Wno-unused-function",
         f"-DTOG_HEADER_HASH=0x{h}LL"]
out = ROOT / "ab_var" / "kuka_helper"
out.mkdir(parents=True, exist_ok=True)
if "--isa" in sys.argv:
    isa = pathlib.Path("/tmp/kuka_isa")
    isa.mkdir(exist_ok=True)
    for tag, extra in (("inline", []), ("helper", ["-DTOG_KUKA_HELPER_F"])):
        subprocess.run(["/opt/rocm/bin/hipcc", *flags, *extra, "--cuda-device-only", "-S", "k_mt_kuka.hip", "-o",
                        str(isa / f"k_mt_kuka_{tag}.s")], cwd=CS, check=True)
    print("listings in", isa)
    sys.exit(0)
subprocess.run(["/opt/rocm/bin/hipcc", *flags, "-DTOG_KUKA_HELPER_F", "-c", "k_mt_kuka.hip", "-o", str(out / "k_mt_kuka.o")],
               cwd=CS, check=True)
objs = [str(CS / o) for o in ["tog_runtime.o", "tog_altro.o", "k_quadrotor_jac.o"]]
models = re.search(r"^MODELS = (.*)$", mk, re.M).group(1).split()
for mname in models:
    objs.append(str(out / "k_mt_kuka.o") if mname == "mt_kuka" else str(CS / f"k_{mname}.o"))
subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "--offload-arch=gfx950", "-fPIC", "-o", str(out / "libtog.so"), *objs],
               check=True)
print("built", out / "libtog.so")
