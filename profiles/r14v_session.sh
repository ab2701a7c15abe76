#!/bin/bash
# Round 6 close: the whole GPU suite with hub-first labels / partition codes forced on every graph (FGI_LABELS=1),
# and the measurement-variant library's suite (libfgi_variants.so: fused waves, probe summary, cooperative cascades)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r14v; mkdir -p $out
cd $R
FGI_LABELS=1 timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $out/labels.log 2>&1
echo "labels rc=$?: $(tail -1 $out/labels.log)"; grep FAILED $out/labels.log | head -5
FGI_LIBRARY=$R/stl.fusion_amd/lib/libfgi_variants.so timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $out/variants.log 2>&1
echo "variants rc=$?: $(tail -1 $out/variants.log)"; grep FAILED $out/variants.log | head -5
exit 0
