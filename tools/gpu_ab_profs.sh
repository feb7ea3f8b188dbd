# gpu_ab.sh on the listed libraries, then tools/gpu_profiles.sh on PROFS
# (space-separated lib.so:ENV=1 entries):
#   PROFS="build/a/lib.so:HL_I4_NAMES=1 ..." bash tools/gpu_ab_profs.sh tag lib1.so [lib2.so ...]
set -o pipefail
tag=$1
bash "$(dirname "$0")/gpu_ab.sh" "$@" || exit 1
bash "$(dirname "$0")/gpu_profiles.sh" ${tag}_prof $PROFS
