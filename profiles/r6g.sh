#!/bin/bash
# Round 6: the full GPU suite and smoke() on the round's HEAD (what the driver runs at round end).
set -o pipefail
O=gpurun_out/r6g
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?
tail -5 $O/tests.log
grep -E "FAILED|ERROR" $O/tests.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
