# round-3 profiles at HEAD: the default command under rocprofv3 (line vs kernel averages), per-config kernel stats, PMC traffic passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
PROF_CONFIGS="rs_enc rs_dec crs_enc crs_dec rs8_small" bash tools/final_prof.sh || exit $?
PROF_CONFIGS="rs_enc rs_dec rs_dec_mixed rs8_small crs_enc crs_dec" bash tools/gpu_session.sh pmc
