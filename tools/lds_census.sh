for T in 0 1; do for G in 512 1024 1280 2048; do
PCORE_LDS_GRANULE=$G PCORE_FUSED_TIER=$T PCORE_LIB=$PWD/build_ab/wgt.so timeout -k 10 100 python tools/wg_timeline.py > gpurun_out/wgt_t${T}_g$G.json 2>gpurun_out/wgt.err || exit 1
echo T$T G$G $(python -c "import json;d=json.load(open('gpurun_out/wgt_t${T}_g$G.json'));print(d['max_concurrency'],round(d['span_us'],1),round(d['dur_mean_us'],1))")
done; done
