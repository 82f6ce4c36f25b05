# Interleaved bench runs of several flag sets (two rounds), one log per run.
# Usage: bash r3_modes.sh tag "flags A" "flags B" ...   ("" = the default pipeline)
# The last flag set also runs once with the parity check on (its _parity.log).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=$1; shift
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --steps 3 --warmup 1"
LAST="${@: -1}"
$B $LAST > gpurun_out/${T}_parity.log 2>&1 || exit 1
for r in 1 2; do
  i=0
  for F in "$@"; do
    $B --no-parity $F > gpurun_out/${T}_m${i}_${r}.log 2>&1 || exit 1
    i=$((i + 1))
  done
done
