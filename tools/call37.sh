# round 4, call 37: end-of-round state -- GPU suite, smoke, the headline bench,
# then the headline bench under a kernel trace (timeline of the final kernels)
set -o pipefail
bash tools/gpu_session.sh tests smoke bench1 prof_bench || exit $?
