# k_pyramid experiments: kernel-trace durations of the two groups under debug switches / tile sizes
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
run() { # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 60 rocprofv3 --kernel-trace -d gpurun_out/exp_$name -o run --output-format csv -- python3 profiles/scripts/extract_only.py 10 > gpurun_out/exp_$name.log 2>&1
}
run base ORBFE_X=0 &&
run skiplevels ORBFE_PYR_DEBUG=1 &&
run nostores ORBFE_PYR_DEBUG=2 &&
run noloads ORBFE_PYR_DEBUG=4 &&
run noloads_nostores ORBFE_PYR_DEBUG=6 &&
run tileA128 ORBFE_PYR_TILE_A=128x32 &&
run tileA32 ORBFE_PYR_TILE_A=32x16 &&
run tileA64x64 ORBFE_PYR_TILE_A=64x64
