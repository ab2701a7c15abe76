mkdir -p gpurun_out/diag
for d in ${DIAGS:-0 1 2 3 4 8 15}; do
  if [ $d = 0 ]; then lib=stl.fusion_amd/lib/libfgi.so; else lib=stl.fusion_amd/lib/diag/libfgi_d$d.so; fi
  timeout -k 10 200 env FGI_TRACE=1 FGI_LIBRARY=$PWD/$lib python bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/diag/d$d.json 2> gpurun_out/diag/d$d.err || exit 1
done
