# small split-K threshold A/B on config 3; config 2 repeated for noise
set -o pipefail
mkdir -p gpurun_out
c3() { env "$@" timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299; }
c3 DV_SMALL_SPLITK_MN=600000 > gpurun_out/ks_c3_600k.log 2>&1 || exit 1
c3 DV_NO_SMALL_SPLITK=1 > gpurun_out/ks_c3_off.log 2>&1 || exit 1
c3 DV_SMALL_SPLITK_MN=300000 > gpurun_out/ks_c3_300k.log 2>&1 || exit 1
c3 DV_SMALL_SPLITK_MN=3000000 > gpurun_out/ks_c3_3m.log 2>&1 || exit 1
for i in 1 2 3; do timeout -k 10 120 python -u bench.py > gpurun_out/ks_c2_$i.log 2>&1 || exit 1; done
timeout -k 10 200 python -u tools/profile_layers.py > gpurun_out/ks_layers_c2.txt 2>&1
