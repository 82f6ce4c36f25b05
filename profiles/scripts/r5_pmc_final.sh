#!/bin/bash
# Round 5 final: PMC passes (HBM traffic of the bench and of the C5 search, wave-time breakdown).
set -o pipefail
bash profiles/scripts/refresh_profiles.sh pmc || exit 1
echo done
