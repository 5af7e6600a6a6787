set -o pipefail
mkdir -p gpurun_out
gcc -O2 -fPIC -shared -o gpurun_out/libfc2_sampler.so scripts/prof/sampler.c -lrt -ldl &&
FC2_LIB_VARIANT=prof FC2_SAMPLE=$PWD/gpurun_out/samples.txt FC2_SAMPLER_LIB=$PWD/gpurun_out/libfc2_sampler.so timeout -k 10 600 python -u scripts/caller_cpu_profile.py 2000000 1.0 > gpurun_out/cprof.json 2> gpurun_out/cprof.err &&
rm -f gpurun_out/libfc2_sampler.so && echo PROF_OK
