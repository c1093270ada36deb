"""ISA facts behind the tail backward kernel's LDS hand-offs (csrc/tog_bwd_quad.hpp tag_store).

    python tools/quad_tag_isa.py > profiles/r5_quad_tag_isa.txt

Compiles k_quadrotor.hip to gfx950 assembly twice -- the tags as wavefront-scope release stores (the
build) and as workgroup-scope ones -- and reports for k_bwd_quad<Quadrotor, 1>:
* that no FLAT store or FLAT atomic appears (every LDS write is a DS instruction, which the LDS unit
  performs in the issuing wave's order, so a tag written after its data is not seen before it);
* the s_waitcnt lgkmcnt(0) the workgroup-scope release adds (one before every tag store).
Exit status 1 if a FLAT store appears."""
import collections
import pathlib
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = pathlib.Path(__file__).resolve().parents[1]
CSRC = ROOT / "trajectoryoptimization.jl-c79d492b-0548-5874-b488-5a62c1d9d0ca_amd" / "csrc"
SYM = "_ZN3tog10k_bwd_quadINS_9QuadrotorELi1EEEvPKNS_10DevProblemENS_10DevBuffersEi"
WAVE = "__ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WAVEFRONT); };"
WG = "__ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP); };"


def body(asm):
    m = re.search("^" + SYM + r":.*?\n(.*?)\.Lfunc_end", asm, re.S | re.M)
    return m.group(1)


def ops(b):
    return collections.Counter(l.split()[0] for l in b.split("\n")
                               if l.startswith("\t") and not l.startswith(("\t.", "\t;")))


def compile_variant(tmp, text):
    d = tmp / "pkg" / "csrc"  # (the sources include ../../include/)
    shutil.copytree(CSRC, d, ignore=shutil.ignore_patterns("*.o", "*.so", "plugins"))
    shutil.copytree(ROOT / "include", tmp / "include")
    (d / "tog_bwd_quad.hpp").write_text(text)
    out = tmp / "k.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950", "-fPIC",
                    "-Wno-unused-function", "-DTOG_HEADER_HASH=0x1LL", "--cuda-device-only", "-S", "-o", str(out),
                    str(d / "k_quadrotor.hip")], check=True, capture_output=True)
    return body(out.read_text())


def main():
    src = (CSRC / "tog_bwd_quad.hpp").read_text()
    if WAVE not in src:
        sys.exit("tog_bwd_quad.hpp: the wavefront-scope tag_store was not found")
    res = {}
    for name, text in (("wavefront", src), ("workgroup", src.replace(WAVE, WG))):
        with tempfile.TemporaryDirectory() as t:
            res[name] = ops(compile_variant(pathlib.Path(t) / "x", text))
    w = res["wavefront"]
    mem = {k: v for k, v in sorted(w.items()) if k.startswith(("flat_", "ds_", "global_", "scratch_", "buffer_"))}
    print(f"k_bwd_quad<Quadrotor, 1> (gfx950), tag_store at wavefront scope: memory instructions {mem}")
    flat_st = {k: v for k, v in w.items() if k.startswith("flat_") and not k.startswith("flat_load")}
    print(f"FLAT stores / atomics: {flat_st or 'none'} (every LDS write is a DS instruction)")
    wc = lambda c: sum(v for k, v in c.items() if k == "s_waitcnt")  # noqa: E731
    print(f"s_waitcnt instructions: wavefront {wc(w)}, workgroup {wc(res['workgroup'])} "
          f"(+{wc(res['workgroup']) - wc(w)}: the lgkmcnt(0) before each tag store)")
    return 1 if flat_st else 0


if __name__ == "__main__":
    sys.exit(main())
