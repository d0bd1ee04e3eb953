set -e
mkdir -p gpurun_out
L="tools/ab/libfwav_old.so tools/ab/libfwav_nb0.so tools/ab/libfwav_nb1.so"
timeout -k 10 250 python -u tools/ab_topk.py $L > gpurun_out/nb_full.log 2>&1
AB_NQ=165376 timeout -k 10 200 python -u tools/ab_topk.py $L > gpurun_out/nb_half.log 2>&1
AB_CFG=cfg3 timeout -k 10 300 python -u tools/ab_topk.py $L > gpurun_out/nb_cfg3.log 2>&1
