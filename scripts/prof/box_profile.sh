# PC samples of the read loop on the box (scripts/caller_cpu_profile.py under scripts/prof/sampler.c):
#   [FC2_SAMPLE_THREAD=1 | FC2_SAMPLE_PROCESS=1] [PROF_READS=N] [PROF_SCALE=S] [PROF_ARGS=--bam] bash scripts/prof/box_profile.sh
# FC2_SAMPLE_THREAD=1 samples only the loop's own thread on its CPU clock (time spent waiting for
# the parse threads is not sampled); FC2_SAMPLE_PROCESS=1 samples every thread on the process's CPU clock.  Needs the -g build: make -C find_circ2_amd/csrc prof
set -o pipefail
mkdir -p gpurun_out
gcc -O2 -fPIC -shared -o gpurun_out/libfc2_sampler.so scripts/prof/sampler.c -lrt -ldl -lpthread &&
FC2_LIB_VARIANT=prof FC2_SAMPLE=$PWD/gpurun_out/samples.txt FC2_SAMPLER_LIB=$PWD/gpurun_out/libfc2_sampler.so timeout -k 10 600 python -u scripts/caller_cpu_profile.py ${PROF_READS:-2000000} ${PROF_SCALE:-1.0} ${PROF_ARGS:-} > gpurun_out/cprof.json 2> gpurun_out/cprof.err &&
rm -f gpurun_out/libfc2_sampler.so && echo PROF_OK
