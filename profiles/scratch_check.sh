# Env / self-play kernel changes (scratch-free select chains, one legality pass per applied step): the
# bit-exact env and self-play tests, then the env (4096 and 2^20 games), det and classic bench lines.
set -o pipefail
O=gpurun_out/scr
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py tests/test_gpu_env_round.py tests/test_gpu_selfplay.py tests/test_gpu_selfplay_classic.py tests/test_gpu_classic.py tests/test_gpu_evaluate.py tests/test_gpu_headline.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python bench.py --workload env --steps 5 --warmup 1 --no-cpu-baseline > $O/env4096.json 2> $O/env4096.err || exit 1
timeout -k 10 200 python bench.py --workload env --batch 1048576 --steps 3 --warmup 1 --no-cpu-baseline > $O/env1m.json 2> $O/env1m.err || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/det.json 2> $O/det.err || exit 1
timeout -k 10 400 python bench.py --workload classic --steps 2 --warmup 1 --no-cpu-baseline > $O/classic.json 2> $O/classic.err || exit 1
for f in env4096 env1m det classic; do python3 -c "import json,sys; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['unit'], d.get('ms_per_step'), d.get('roofline',{}).get('frac'))"; done
