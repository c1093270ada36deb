"""Extract the iLQR/AL iteration log of the reference's Kuka notebook
(examples/kuka_iiwa/Kuka iiwa.ipynb, cell 16 output: solve!(prob, opts_al)) into
tests/golden/kuka_notebook_log.json. Data only (the printed numbers); run here, where
/root/reference exists, output committed."""
import json
import pathlib
import re

NB = pathlib.Path("/root/reference/examples/kuka_iiwa/Kuka iiwa.ipynb")
OUT = pathlib.Path(__file__).resolve().parent / "kuka_notebook_log.json"

nb = json.loads(NB.read_text())
text = "".join(o.get("text", "") if isinstance(o.get("text", ""), str) else "".join(o["text"])
               for o in nb["cells"][16]["outputs"])
text = re.sub(r"\x1b\[[0-9;]*m", "", text)
inner, outer = [], []
for line in text.splitlines():
    f = line.split()
    if len(f) == 9 and re.fullmatch(r"\d+", f[0]):  # iter cost expected z α ρ dJ grad zero_count
        inner.append({"cost": float(f[1]), "expected": float(f[2]), "z": float(f[3]), "alpha": float(f[4]),
                      "dJ": float(f[6]), "grad": float(f[7])})
    elif len(f) == 4 and re.fullmatch(r"\d+", f[0]) and re.fullmatch(r"\d+", f[1]):  # iter total c_max cost
        outer.append({"iter": int(f[0]), "total": int(f[1]), "c_max": float(f[2]), "cost": float(f[3])})
OUT.write_text(json.dumps({"source": "examples/kuka_iiwa/Kuka iiwa.ipynb cell 16", "inner": inner,
                           "outer": outer}, indent=1))
print(f"{len(inner)} inner, {len(outer)} outer rows -> {OUT}")
