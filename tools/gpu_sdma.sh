#!/bin/bash
# A/B: large D2H copies by SDMA engines (HSA_ENABLE_SDMA=1) vs the runtime default (blit kernels
# in the kernel trace), alternating, 60 steps each; plus a kernel trace with SDMA on.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/sdma; mkdir -p $O
for i in 1 2; do
  for v in default 1; do
    if [ $v = default ]; then
      timeout -k 10 300 python bench.py --steps 60 --warmup 5 > $O/h_${v}_$i.log 2>&1 || exit $?
    else
      HSA_ENABLE_SDMA=$v timeout -k 10 300 python bench.py --steps 60 --warmup 5 > $O/h_${v}_$i.log 2>&1 || exit $?
    fi
    python3 -c "
import json
d=json.loads([l for l in open('$O/h_${v}_$i.log') if l.startswith('{')][-1]); s=d['stage_ms_per_step']
print('sdma=$v', round(d['value']/1e6,1), d['ms_per_step'], 'join', s['t_join_ms'], 'out', s['t_out_ms'], 'parse', s['t_parse_ms'])"
  done
done
HSA_ENABLE_SDMA=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || exit $?
echo prof ok
