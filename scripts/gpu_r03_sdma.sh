# Does GPU_FORCE_BLIT_COPY_SIZE=0 move D2H copies off the blit kernels onto the DMA engines?  The copy
# probe with the runtime's copy log, then the strong-scaling repetitions under that setting.
set -o pipefail
mkdir -p gpurun_out/sdma
GPU_FORCE_BLIT_COPY_SIZE=0 AMD_LOG_LEVEL=3 timeout -k 10 200 python -u scripts/probes/copy_engine_probe.py > gpurun_out/sdma/log3.out 2>&1 && echo LOG_OK &&
(grep -c 'HSA Copy' gpurun_out/sdma/log3.out || true) &&
(grep -c 'ShaderName : __amd_rocclr_copyBuffer' gpurun_out/sdma/log3.out || true) &&
(grep -m 5 'HSA Copy' gpurun_out/sdma/log3.out || true) &&
(grep '^{' gpurun_out/sdma/log3.out | tail -1 > gpurun_out/sdma/probe.json || true) && rm -f gpurun_out/sdma/log3.out &&
GPU_FORCE_BLIT_COPY_SIZE=0 REPEAT=9 timeout -k 10 900 python -u scripts/probes/strong_streams_probe.py > gpurun_out/sdma/strong_repeat.jsonl 2> gpurun_out/sdma/strong_repeat.err && echo REPEAT_OK &&
cat gpurun_out/sdma/probe.json gpurun_out/sdma/strong_repeat.jsonl
