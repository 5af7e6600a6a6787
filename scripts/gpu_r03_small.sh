set -o pipefail
mkdir -p gpurun_out/small
for v in count esc; do
  FC2_STRONG_SMALL_LAST=$v REPEAT=9 timeout -k 10 800 python -u scripts/probes/strong_streams_probe.py > gpurun_out/small/$v.jsonl 2> gpurun_out/small/$v.err || exit 1
  echo "== $v"; cut -c1-100 gpurun_out/small/$v.jsonl
done
