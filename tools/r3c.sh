set -u
bash tools/r3a.sh || exit $?
bash tools/r3b.sh
