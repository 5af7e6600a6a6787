# The configs[3] merge's copy/scan overlap against the stream choice, at HIP's default 4 hardware
# queues per process and at 8 and 16 (scripts/probes/strong_streams_probe.py).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/strong_streams.jsonl
for q in 4 8 16; do
  echo "{\"GPU_MAX_HW_QUEUES\": $q}" >> gpurun_out/strong_streams.jsonl
  GPU_MAX_HW_QUEUES=$q timeout -k 10 600 python -u scripts/probes/strong_streams_probe.py >> gpurun_out/strong_streams.jsonl 2>> gpurun_out/strong_streams.err || exit 1
done
echo PROBE_OK
cat gpurun_out/strong_streams.jsonl
