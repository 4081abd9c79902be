cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04_codec
for r in 8 16; do
  timeout -k 10 400 python bench.py --workload c5z --steps 10 --warmup 2 --no-cpu --no-c3 --no-next-row --e2e-dev-ranges $r > gpurun_out/r04_codec/bench_c5z_r$r.log 2>&1 || exit $?
done
