# Version 4 timing ablations at the Syn-10M shard (results invalid by construction): abl4 = LDS-DMA issued but
# never waited for in the loop, abl1 = no LDS-DMA and no waits; alternating processes with the default. Then
# the LDS bank-conflict census (scripts/gpu_r02s3_ldsconf.sh).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abl4
mkdir -p $O
cd $R
for i in 1 2; do
  timeout -k 10 200 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 6 --rounds 1 > $O/base_$i.jsonl 2>&1
  HVAE_LIB=$R/build_var/libhvae_abl4.so timeout -k 10 200 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 6 --rounds 1 > $O/abl4_$i.jsonl 2>&1
  HVAE_LIB=$R/build_var/libhvae_abl1.so timeout -k 10 200 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 6 --rounds 1 > $O/abl1_$i.jsonl 2>&1
done
bash $R/scripts/gpu_r02s3_ldsconf.sh
