"""The Julia binding's struct mirrors (integration/julia/libtog.jl) against include/tog.h.

No Julia here, so two checks stand in for its own `tog_check_layout()`:
* the layout constants libtog.jl asserts at run time (TOG_LAYOUT, TOG_DESC_OFFSETS, TOG_ABI_VERSION) equal
  sizeof / offsetof / TOG_ABI_VERSION of the C structs, compiled here by gcc from include/tog.h;
* the field lists of the Julia structs, laid out with Julia's C-compatible rules (natural alignment, isbits
  structs inline), give the same sizes and offsets, field by field, as the C structs."""
import pathlib
import re
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
JL = (ROOT / "integration" / "julia" / "libtog.jl").read_text()

STRUCTS = {  # Julia mirror -> C struct
    "TogConstraint": "tog_constraint", "TogConstraintSet": "tog_constraint_set", "TogProblemDesc": "tog_problem_desc",
    "TogOptionsI": "tog_options", "TogPNOptions": "tog_pn_options", "TogAltroOptions": "tog_altro_options",
    "TogAltroResult": "tog_altro_result",
}
PRIM = {"Int32": (4, 4), "Int64": (8, 8), "Float64": (8, 8), "Cvoid": None}


def julia_fields(name):
    m = re.search(r"^(?:mutable )?struct " + name + r"\b[^\n]*\n(.*?)^end", JL, re.S | re.M)
    assert m, name
    body = m.group(1).split("function")[0]
    fields = []
    for part in re.split(r"[;\n]", body):
        part = part.split("#")[0].strip()
        if "::" in part:
            f, t = part.split("::")
            fields.append((f.strip(), t.strip()))
    return fields


def julia_layout(name):
    off, align = 0, 1
    offsets = []
    for f, t in julia_fields(name):
        if t.startswith("Ptr{"):
            size, al = 8, 8
        elif t in PRIM:
            size, al = PRIM[t]
        else:
            size, al = julia_layout(t)[0], 8
        off = (off + al - 1) // al * al
        offsets.append((f, off))
        off += size
        align = max(align, al)
    return (off + align - 1) // align * align, offsets


@pytest.fixture(scope="module")
def c_layout(tmp_path_factory):
    d = tmp_path_factory.mktemp("layout")
    lines = ['#include <stddef.h>', '#include <stdio.h>', '#include "tog.h"', "int main(void) {",
             'printf("abi %d\\n", TOG_ABI_VERSION);']
    for jl, c in STRUCTS.items():
        lines.append(f'printf("size {c} %zu\\n", sizeof({c}));')
        for f, _ in julia_fields(jl):
            lines.append(f'printf("off {c} {f} %zu\\n", offsetof({c}, {f}));')
    lines += ["return 0;", "}"]
    (d / "l.c").write_text("\n".join(lines))
    subprocess.run(["gcc", "-I", str(ROOT / "include"), str(d / "l.c"), "-o", str(d / "l")], check=True)
    out = subprocess.run([str(d / "l")], capture_output=True, text=True, check=True).stdout.split("\n")
    res = {"size": {}, "off": {}}
    for ln in out:
        p = ln.split()
        if not p:
            continue
        if p[0] == "abi":
            res["abi"] = int(p[1])
        elif p[0] == "size":
            res["size"][p[1]] = int(p[2])
        else:
            res["off"][(p[1], p[2])] = int(p[3])
    return res


def test_julia_pinned_constants_match_c(c_layout):
    assert int(re.search(r"const TOG_ABI_VERSION = Int32\((\d+)\)", JL).group(1)) == c_layout["abi"]
    pins = dict(re.findall(r"(tog_\w+) = (\d+)", re.search(r"const TOG_LAYOUT = \((.*?)\)\n", JL, re.S).group(1)))
    for c in STRUCTS.values():
        assert int(pins[c]) == c_layout["size"][c], c
    offs = [int(v) for v in re.search(r"const TOG_DESC_OFFSETS = \((.*?)\)\n", JL, re.S).group(1).replace("\n", " ").split(",")]
    assert offs == [c_layout["off"][("tog_problem_desc", f)] for f, _ in julia_fields("TogProblemDesc")]


@pytest.mark.parametrize("jl", list(STRUCTS))
def test_julia_struct_fields_lay_out_like_c(c_layout, jl):
    c = STRUCTS[jl]
    size, offsets = julia_layout(jl)
    assert size == c_layout["size"][c]
    for f, off in offsets:
        assert off == c_layout["off"][(c, f)], (c, f)
