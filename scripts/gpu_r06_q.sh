# Round 6, call Q: the CSR catch-up with four column groups' loads in flight per thread (HVAE_CATCHUP_UNROLL=4 in
# the A/B library) against one (the product's), alternating, at Syn-1M and the fp8 Syn-10M shard.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06q
mkdir -p $O
cd $R
ab() {  # unroll workload precision
  HVAE_LIB=build_var/libhvae_ab.so HVAE_CATCHUP_UNROLL=$1 timeout -k 10 300 python -u bench.py --workload $2 --precision $3 \
    --steps 150 --warmup 30 --no-cpu-baseline --probe-steps 2 2>> $O/bench.err | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'catchup_unroll':$1,'workload':'$2','precision':'$3','ms':d['ms_per_step'],'catchup_us':d['launch_us']['adam_catchup']['avg_us']}))" >> $O/catchup_unroll_ab.jsonl || exit 2
}
for r in 1 2; do
  for u in 1 4; do ab $u syn1m bf16; done
  for u in 1 4; do ab $u syn10m fp8; done
done
echo done > $O/done
