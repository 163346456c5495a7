set -o pipefail
export DV_ABLATIONS=1  # the A/B switches below are honoured only in ablation mode (knobs.py)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_deepdream.py -m gpu -k "octave or fused or split" > gpurun_out/dd_tests.log 2>&1 && \
for i in 1 2 3; do
  DV_DREAM_OCTAVE_RESIZE=0 timeout -k 10 200 python bench_dream.py --runs 3 >> gpurun_out/c3_ab.log 2>&1 && echo "^old" >> gpurun_out/c3_ab.log && \
  DV_DREAM_OCTAVE_RESIZE=1 timeout -k 10 200 python bench_dream.py --runs 3 >> gpurun_out/c3_ab.log 2>&1 && echo "^new" >> gpurun_out/c3_ab.log || exit 1
done
