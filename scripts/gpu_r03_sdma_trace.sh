# Which engine runs the D2H copies with GPU_FORCE_BLIT_COPY_SIZE=0: kernel + memory-copy trace of the copy probe.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/sdma
export TMPDIR=/tmp && cd /tmp &&
GPU_FORCE_BLIT_COPY_SIZE=0 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/sdma/trace -o tr --output-format csv -- python3 $R/scripts/probes/copy_engine_probe.py > $R/gpurun_out/sdma/trace.out 2>&1 && echo TRACE_OK
ls $R/gpurun_out/sdma/trace
