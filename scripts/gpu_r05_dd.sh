# Lazy-Adam sweep period 32 (product) vs 48 / 64 (variant libraries built with -DHVAE_LAZY_SWEEP) at Syn-10M and
# Syn-1M: per-step time and the adam_rows / adam_catchup launch averages, two interleaved rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r05dd
mkdir -p $O
for round in 1 2; do
  for wl in syn10m syn1m; do
    for a in base sweep48 sweep64; do
      lib=$R/build_var/libhvae_$a.so; [ $a = base ] && lib=$R/recommendation-system_amd/hvae/libhvae.so
      HVAE_LIB=$lib timeout -k 10 240 python -u bench.py --workload $wl --steps 30 --warmup 10 --no-cpu-baseline \
        > $O/bench_${wl}_$a.json 2>> $O/bench.log || exit 4
      python3 -c "
import json; d=json.loads(open('$O/bench_${wl}_$a.json').read().strip().split(chr(10))[-1]); L=d['launch_us']
print(json.dumps({'arm': '$a', 'workload': '$wl', 'round': $round, 'ms_per_step': d['ms_per_step'], 'adam_rows_us': L['adam_rows']['avg_us'], 'adam_catchup_us': L['adam_catchup']['avg_us'], 'sweep_us': L['decoder_sweep']['avg_us']}))" >> $O/sweep_period.jsonl
    done
  done
done
cat $O/sweep_period.jsonl
