# is config 3 host-bound on hipGraph launches? host enqueue time vs wall, split 1/2, packet capture on/off
set -o pipefail
mkdir -p gpurun_out
run() { tag=$1; shift; env "$@" timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/hb_$tag.log 2>&1; }
run s2 DV_DREAM_SPLIT=2 || exit 1
run s1 DV_DREAM_SPLIT=1 || exit 1
run s2_pc1 DV_DREAM_SPLIT=2 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 || exit 1
run s2_pc0 DV_DREAM_SPLIT=2 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit 1
run s4_pc1 DV_DREAM_SPLIT=4 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 || exit 1
run s2_bs64 DV_DREAM_SPLIT=2 DEBUG_HIP_GRAPH_BATCH_SIZE=64 || exit 1
