#!/bin/bash
# kres.sh <model.hip> <kernel-substring> [extra hipcc flags...]: VGPR/AGPR/scratch/occupancy per kernel
f=$1; pat=$2; shift 2
cd "$(dirname "$0")/../trajectoryoptimization.jl-c79d492b-0548-5874-b488-5a62c1d9d0ca_amd/csrc" || exit 1
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -fPIC "$@" -c "$f" -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import sys,re
pat=sys.argv[1]; cur=None; out={}
keys={"VGPRs:":"vgpr","AGPRs:":"agpr","ScratchSize [bytes/lane]:":"scratch","Occupancy [waves/SIMD]:":"occ","LDS Size [bytes/block]:":"lds"}
for l in sys.stdin:
    m=re.search(r"Function Name: (\S+)",l)
    if m:
        cur=m.group(1) if pat in m.group(1) else None
        continue
    if cur:
        for k,v in keys.items():
            if k in l: out.setdefault(cur,[]).append(v+"="+l.split(k)[1].split()[0])
for k in sorted(out): print(k[:64], " ".join(out[k]))
' "$pat"
