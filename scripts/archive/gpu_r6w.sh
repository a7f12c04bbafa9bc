# batches in flight (depth) A/B for C3 and C2 (interleaved, two rounds)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6w
mkdir -p $OUT
for rep in 1 2; do
  for dp in 3 4 5; do
    timeout -k 10 200 python bench.py --mixed --steps 20 --warmup 3 --depth $dp --no-cpu-baseline --no-extras > $OUT/c3_d${dp}_$rep.json 2> $OUT/c3_d${dp}_$rep.err || exit $?
    timeout -k 10 200 python bench.py --steps 40 --warmup 5 --depth $dp --no-cpu-baseline --no-extras > $OUT/c2_d${dp}_$rep.json 2> $OUT/c2_d${dp}_$rep.err || exit $?
    python -c "
import json
a=json.loads(open('$OUT/c3_d${dp}_$rep.json').read().strip().splitlines()[-1]); b=json.loads(open('$OUT/c2_d${dp}_$rep.json').read().strip().splitlines()[-1])
print('depth $dp rep $rep', 'C3', a['value'], 'C2', b['value'], flush=True)"
  done
done
