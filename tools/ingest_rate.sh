#!/bin/bash
# Step 0 + prepare rate on a config-E FASTA (CPU only, no GPU): tools/synth_fa
# writes N ZMWs, tools/ubench/ingest_bench reads and groups them (one reader
# thread, as the CLI's step 0) and assembles + prepares them on T threads.
#   bash tools/ingest_rate.sh N T OUTDIR
set -e
N=${1:-200000}; T=${2:-16}; OUT=${3:-gpurun_out/ingest}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/$OUT"
F=$(mktemp -d ${TMPDIR:-/tmp}/ccsx_ingest_XXXX)/e.fa
"$R/tools/synth_fa" "$N" 20000000 0 0 "$T" > "$F"
timeout -k 10 600 "$R/tools/ubench/ingest_bench" "$F" 0 "$T" 16384 > "$R/$OUT/ingest_${N}_t$T.json"
cat "$R/$OUT/ingest_${N}_t$T.json"
rm -f "$F"; rmdir "$(dirname "$F")"
