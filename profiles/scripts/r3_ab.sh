# A/B of the in-tree library against lib/alt: extraction alone (extract_only.py --per-kernel, the bench's
# driving-sequence frames), then the bench line, interleaved. Usage: bash r3_ab.sh [tag] [extra bench flags]
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-ab}; shift || true
ALT=orb_slam2_2021_amd/lib/alt/liborbfe.so
X="timeout -k 10 120 python profiles/scripts/extract_only.py 20 --per-kernel --seq"
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 3 --warmup 1 $*"
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_test.log 2>&1 &&
$X > gpurun_out/${T}_xnew1.log 2>&1 && ORBFE_LIB=$ALT $X > gpurun_out/${T}_xold1.log 2>&1 &&
$X > gpurun_out/${T}_xnew2.log 2>&1 && ORBFE_LIB=$ALT $X > gpurun_out/${T}_xold2.log 2>&1 &&
$B > gpurun_out/${T}_bnew1.log 2>&1 && ORBFE_LIB=$ALT $B > gpurun_out/${T}_bold1.log 2>&1 &&
$B > gpurun_out/${T}_bnew2.log 2>&1 && ORBFE_LIB=$ALT $B > gpurun_out/${T}_bold2.log 2>&1
