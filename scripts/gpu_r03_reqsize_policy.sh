# Request sizes of random 16/32-B gathers under every allocation type and cache policy
# (scripts/policy_probe.hip): does any form leave L2 as a request smaller than 128 B?
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/req_policy
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 $R/scripts/policy_probe > $OUT/policy_probe.json 2> $OUT/policy_probe.err && echo PLAIN_OK &&
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d $OUT/sizes -o pmc --output-format csv -- $R/scripts/policy_probe > $OUT/sizes.out 2>&1 && echo SIZES_OK &&
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum -d $OUT/dram -o pmc --output-format csv -- $R/scripts/policy_probe > $OUT/dram.out 2>&1 && echo DRAM_OK
