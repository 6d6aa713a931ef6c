# Row-parallel MLP launch times against the layer widths at B = 64 (which layer's weight stream costs what).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_mlp_shapes}
mkdir -p $O
cd $R
timeout -k 10 200 python scripts/bench_mlp_rows.py --batches 64 --shapes 512:128:384,512:128:32,512:32:384,32:32:384,32:128:384,32:32:32,512:128:768,256:128:384 > $O/shapes.jsonl 2> $O/shapes.err
