#!/bin/bash
# round 5: the whole GPU suite on the current tree, then smoke
set -o pipefail
O=gpurun_out/${SUITE_OUT:-r05suite}; mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 650 --timeout-method thread > $O/pytest.log 2>&1 || { echo "suite failed"; grep -E "FAILED|Error" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -n 3 $O/smoke.log
