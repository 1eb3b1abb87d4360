set -u
for t in 8 16 8 16 8 16; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --join-threads $t > gpurun_out/ab.log 2>&1 || exit $?; echo "threads=$t $(tail -1 gpurun_out/ab.log | cut -c60-150)"
done
