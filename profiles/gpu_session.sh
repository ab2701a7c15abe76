#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench, rocprof evidence. Stops at the first crash-like
# exit (fault/abort/segv/timeout); an ordinary test failure (pytest exit 1) still lets the bench run.
# Usage (from the repo root, on the box): profiles/gpu_session.sh <tag> [pytest selection]
#   SKIP_TESTS=1 / SKIP_BENCH=1 / SKIP_PROFILE=1 skip those steps.
TAG=${1:-r02}
SEL=${2:-tests}
O=gpurun_out/$TAG
mkdir -p "$O"
crash() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
    timeout -k 10 900 python -u -m pytest $SEL -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread \
        > "$O/gpu_tests.log" 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 "$O/gpu_tests.log"; crash $rc && exit $rc
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit 21
    echo "smoke ok"
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
    timeout -k 10 500 python bench.py $BENCH_ARGS > "$O/bench.json" 2> "$O/bench.err" || exit 22
    cat "$O/bench.json"
fi
[ "${SKIP_PROFILE:-1}" = 1 ] && exit 0
profiles/run_profile.sh "$TAG" || exit 23
