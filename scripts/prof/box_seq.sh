# The sequential read loop on the box (scripts/caller_cpu_profile.py, oracle behind the batch hook):
# seconds in next / submit per 2M reads on the hg19-sized genome, twice.
set -o pipefail
mkdir -p gpurun_out
for k in 1 2; do
  timeout -k 10 300 python -u scripts/caller_cpu_profile.py 2000000 1.0 > gpurun_out/seq_$k.json 2>> gpurun_out/seq.err || exit 1
  cat gpurun_out/seq_$k.json
done
