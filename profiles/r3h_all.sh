#!/bin/bash
# Round-3 final check: full GPU suite + smoke + headline profile (r3h_validate.sh), then the env micro-benchmark at
# 4096 and 2^20 games and env_breakdown.py.
set -o pipefail
bash profiles/r3h_validate.sh || exit 1
O=gpurun_out/r3h
timeout -k 10 200 python bench.py --workload env --steps 5 --warmup 1 --cpu-seconds 10 > $O/env_4096.json 2> $O/env_4096.err || { tail -20 $O/env_4096.err; exit 1; }
timeout -k 10 200 python bench.py --workload env --batch 1048576 --steps 3 --warmup 1 --no-cpu-baseline > $O/env_1m.json 2> $O/env_1m.err || { tail -20 $O/env_1m.err; exit 1; }
timeout -k 10 200 python profiles/env_breakdown.py > $O/env_breakdown.log 2>&1 || { tail -20 $O/env_breakdown.log; exit 1; }
python3 -c "
import json
for n in ('env_4096', 'env_1m'):
    d = json.load(open('$O/' + n + '.json')); r = d['roofline']; print(n, d['value'], r['kernel'], r['avg_launch_ms'], r['frac'])"
grep "B=" $O/env_breakdown.log
