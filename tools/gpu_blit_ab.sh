#!/bin/bash
# config 2: the mosaics' D2H copy runs as a 256-workgroup blit kernel (__amd_rocclr_copyBuffer, 2.8 ms) next to the
# next step's compute; A/B of HIP runtime settings that shrink it or move it off the CUs
set -o pipefail
O=gpurun_out/blitab
mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 150 python bench.py --steps 20 --warmup 3 > $O/$n.json 2>$O/$n.err || exit 1
}
for r in 1 2; do
  run base_$r DV_NOP=1
  run wg8_$r DEBUG_CLR_LIMIT_BLIT_WG=8
  run wg32_$r DEBUG_CLR_LIMIT_BLIT_WG=32
  run sdma_$r HSA_ENABLE_SDMA=1
done
