set -e
mkdir -p gpurun_out
B=scripts/bench_decoder.py
for N in 320 1600 6400 12101 50000; do
  timeout -k 10 120 python $B --nb 64 --N $N --D 384 --reps 50 2>&1 | grep -v amdgpu.ids >> gpurun_out/dec_small.log
done
timeout -k 10 120 python $B --nb 64 --N 12101 --D 384 --reps 50 --train --probe decoder_finalize 2>&1 | grep -v amdgpu.ids >> gpurun_out/dec_small.log
timeout -k 10 120 python $B --nb 64 --N 12101 --D 384 --reps 50 --train 2>&1 | grep -v amdgpu.ids >> gpurun_out/dec_small.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_dec -o run -- python3 $GRAFT_REPO_ROOT/$B --nb 64 --N 12101 --D 384 --reps 50 --train > $GRAFT_REPO_ROOT/gpurun_out/prof_dec.log 2>&1
