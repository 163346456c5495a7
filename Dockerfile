# MI355X (gfx950) image for the deconvnet service. The reference's image is python:3.7 + CPU
# TensorFlow running `uvicorn main:app --port 80` (reference Dockerfile:1-15); this one builds the
# HIP kernels in-tree and starts one GPU-owner process per visible GPU; each rank runs DV_FRONTENDS HTTP
# front ends on port 80 (SO_REUSEPORT, under a per-rank supervisor that restarts a dead one).
# pinned base: ROCm 7.2 + PyTorch 2.10 (rocm7.0 wheel), Python 3.10 -- the stack this tree is tested on
FROM rocm/pytorch:rocm7.2_ubuntu22.04_py3.10_pytorch_release_2.10.0

ENV HSA_ENABLE_IPC_MODE_LEGACY=0 \
    PYTORCH_ROCM_ARCH=gfx950 \
    DV_PORT=80
WORKDIR /app
COPY requirements.txt /app/
RUN pip install --no-cache-dir -r requirements.txt
COPY . /app
RUN python -m deconv_api_amd._build --force

EXPOSE 80
CMD ["python", "-m", "torch.distributed.run", "--standalone", "--nproc-per-node", "gpu", \
     "-m", "deconv_api_amd.serve.launch"]
