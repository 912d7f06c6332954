# round 4: which pass in front of K2 makes it fast? (policy of a 256 MiB pass over another buffer)
set -o pipefail
M="1:0,18:256,19:256,20:256,30:256,21:256,31:256,22:256,32:256,23:256,33:256,23:1024,33:1024,0:0,7:0"
EXP_LIB=../ab_exp/libexp_k1k2.so EXP_CFG=cfg3 EXP_MODES=$M timeout -k 10 300 python tools/exp_k1k2.py 2 10 > gpurun_out/r04_k2pass_cfg3.json 2> gpurun_out/r04_k2pass_cfg3.err || exit 1
cat gpurun_out/r04_k2pass_cfg3.json
EXP_LIB=../ab_exp/libexp_k1k2.so EXP_CFG=cfg2 EXP_MODES=$M timeout -k 10 300 python tools/exp_k1k2.py 2 40 > gpurun_out/r04_k2pass_cfg2.json 2> gpurun_out/r04_k2pass_cfg2.err || exit 1
cat gpurun_out/r04_k2pass_cfg2.json
