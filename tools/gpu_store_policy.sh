# k_scan1f block-store cache policy and pipelining study, configs 2 and 3 (tools/tune_fused.py)
set -e
timeout -k 10 240 python tools/tune_fused.py --ks 1 --variants 6,7,8,9,10,11,12,13,14,15,0 --rounds 10 > gpurun_out/tune_policy_c2.log 2>&1
timeout -k 10 300 python tools/tune_fused.py --size-mib 1024 --block-size 1024 --density 0.0099 --ks 2 --variants 6,7,8,9,10,11,12,13,14,15 --rounds 8 > gpurun_out/tune_policy_c3.log 2>&1
