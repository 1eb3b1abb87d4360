#!/bin/bash
# Isolated kernel times (AMD_SERIALIZE_KERNEL=3): headline and audit-heavy (25 %) shards.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ser; mkdir -p $O
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/head -o run -- python3 bench.py --steps 10 --warmup 3 > $O/head.log 2>&1 || exit $?
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/aud25 -o run -- python3 bench.py --steps 10 --warmup 3 --audit-fraction 0.25 > $O/aud25.log 2>&1 || exit $?
echo done
