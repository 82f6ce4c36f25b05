# k_fast workgroup size: waves per workgroup for the side-stream launches (ORBFE_FAST_WPB) and the
# levels-3..7 launch (ORBFE_FAST_WPB_MAIN); extraction alone and the bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
X="timeout -k 10 120 python profiles/scripts/extract_only.py 20 --per-kernel --seq"
B="timeout -k 10 200 python bench.py --no-cpu --no-legs --no-parity --steps 3 --warmup 1"
for m in 1 2 4; do ORBFE_FAST_WPB_MAIN=$m $X > gpurun_out/wpm_x$m.log 2>&1 || exit 1; done &&
for r in 1 2; do for m in 1 2 4; do ORBFE_FAST_WPB_MAIN=$m $B > gpurun_out/wpm_b${m}_$r.log 2>&1 || exit 1; done; done
