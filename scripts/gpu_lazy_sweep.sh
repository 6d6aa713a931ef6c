# Lazy-Adam rotating sweep period A/B (8 = shipped, 16, 32): the bitwise lazy-vs-dense tests on each build, then
# the Syn-10M bench (adam_rows / adam_catchup probes and users/s) per build, two rounds.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/sweep
mkdir -p $O
for v in 16 32; do
  HVAE_LIB=$R/build_var/libhvae_sweep$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -q -k lazy --timeout 200 --timeout-method thread > $O/t_$v.log 2>&1
done
for r in 1 2; do
for v in 8 16 32; do
  if [ $v = 8 ]; then L=""; else L="HVAE_LIB=$R/build_var/libhvae_sweep$v.so"; fi
  env $L timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --probe-steps 5 --no-cpu-baseline > $O/b_$v.json 2> $O/b_$v.err && python -c "import json,sys; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); print(json.dumps({'period': $v, 'value': d['value'], 'ms': d['ms_per_step'], 'adam_rows_us': d['launch_us']['adam_rows']['us_per_step'], 'catchup_us': d['launch_us']['adam_catchup']['us_per_step']}))" >> $O/all.jsonl
done
done
