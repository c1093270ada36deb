#!/bin/bash
# kstats.sh <model> [kernel-substring] [extra hipcc flags]: registers, spills and scratch of one model's kernels
m=${1:-quadrotor}; pat=${2:-k_bwd_team}; shift 2
src="$(cd "$(dirname "$0")/.." && pwd)/trajectoryoptimization.jl-c79d492b-0548-5874-b488-5a62c1d9d0ca_amd/csrc"
d=/tmp/kstats; mkdir -p $d
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -fPIC -gline-tables-only "$@" -c "$src/k_$m.hip" -o $d/x.o -save-temps=obj 2>&1 | grep -E "error" 
python3 - $d/k_$m-hip-amdgcn-amd-amdhsa-gfx950.s "$pat" <<'PY'
import sys,re
s=open(sys.argv[1]).read()
for blk in s.split('  - .agpr_count')[1:]:
    name=re.search(r'\.name:\s+(\S+)',blk).group(1)
    if sys.argv[2] not in name: continue
    g=lambda k: (re.search(r'\.'+k+r':\s+(\d+)',blk) or [0,'?'])[1]
    print(f"{name[:70]:70s} vgpr={g('vgpr_count')} vspill={g('vgpr_spill_count')} sgpr={g('sgpr_count')} sspill={g('sgpr_spill_count')} scratch={g('private_segment_fixed_size')} lds={g('group_segment_fixed_size')}")
PY
