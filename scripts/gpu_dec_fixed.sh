set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for N in 32 320 3200 12101; do
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pdec_$N -o run -- python3 $R/scripts/bench_decoder.py --nb 64 --N $N --D 384 --reps 30 > $R/gpurun_out/pdec_$N.log 2>&1
done
