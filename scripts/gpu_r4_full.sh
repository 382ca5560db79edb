#!/bin/bash
# Round-end rehearsal: every GPU test, smoke(), and the headline bench with the driver's defaults.
source "$(dirname "$0")/gpu_lib.sh"
step gpu_tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 600 python bench.py
exit $status
