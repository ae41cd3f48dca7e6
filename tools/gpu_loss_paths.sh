cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06o
OUT=gpurun_out/r06o
run() { tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --fresh-rays 0 "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo $tag failed; tail -5 $OUT/$tag.err; exit 4; }; python -c "
import json; d=json.loads(open('$OUT/$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d.get('loss'), d.get('fused_table_step'))"; }
run plain
run plain2
run nofuse --fused-table-step 0
run det --deterministic 1
run det_nofuse --deterministic 1 --fused-table-step 0
run nograph --graph 0
run nograph_nofuse --graph 0 --fused-table-step 0
