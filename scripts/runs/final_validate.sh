#!/bin/bash
# end-of-round validation at HEAD: build check, smoke, the whole GPU test suite (one process, per-test timeouts)
set -o pipefail
O=${1:-gpurun_out/final6}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.build(); g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputest.log 2>&1 || exit 1
