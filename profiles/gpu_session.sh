#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench, rocprof evidence. Stops at the first crash-like
# exit (fault/abort/segv/timeout); an ordinary test failure (pytest exit 1) still lets the bench run.
# Usage (from the repo root, on the box): profiles/gpu_session.sh <tag>
TAG=${1:-r02}
O=gpurun_out/$TAG
mkdir -p "$O"
crash() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
timeout -k 10 700 python -m pytest tests -m gpu -q -p no:cacheprovider > "$O/gpu_tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; crash $rc && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit 21
echo "smoke ok"
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err" || exit 22
cat "$O/bench.json"
[ "${SKIP_PROFILE:-0}" = 1 ] && exit 0
profiles/run_profile.sh "$TAG" || exit 23
