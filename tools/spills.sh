#!/bin/bash
# spills.sh <model.hip> <kernel-substring> [flags]: scratch stores per source line of one kernel
f=$1; pat=$2; shift 2
cd "$(dirname "$0")/../trajectoryoptimization.jl-c79d492b-0548-5874-b488-5a62c1d9d0ca_amd/csrc" || exit 1
d=$(mktemp -d)
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -fPIC -gline-tables-only "$@" -c "$f" -o $d/x.o -save-temps=obj 2>/dev/null
python3 - $d/*gfx950*.s "$pat" <<'PY'
import re,sys,collections
s=open(sys.argv[1]).read().split('\n'); pat=sys.argv[2]
starts=[i for i,l in enumerate(s) if re.match(r'^_Z\S*:',l) and pat in l]
for a in starts:
    b=a+1
    while not s[b].startswith('.Lfunc_end'): b+=1
    st=collections.Counter(); ld=collections.Counter(); cur=None
    for l in s[a:b]:
        if l.strip().startswith('.loc'):
            m=re.findall(r'tog_bwd_team.hpp:(\d+)',l)
            if m: cur=int(m[-1]) if '@[' not in l else int(m[-1])
        if 'scratch_store' in l: st[cur]+=1
        if 'scratch_load' in l: ld[cur]+=1
    print(s[a].split(':')[0][:60], 'stores', sum(st.values()), 'loads', sum(ld.values()))
    print('  top store lines', st.most_common(8))
    print('  top load lines', ld.most_common(8))
PY
rm -rf $d
