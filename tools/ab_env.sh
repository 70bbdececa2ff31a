# Alternate full bench.py runs between two environment settings on one box (A B A B ...).
#   bash tools/ab_env.sh "ENV_A" "ENV_B" ROUNDS OUTDIR [bench args...]
set -e
A=$1; B=$2; R=$3; OUT=$4; shift 4
mkdir -p $OUT
for r in $(seq 1 $R); do
  env $A timeout -k 10 200 python3 bench.py --no-cpu-baseline "$@" > $OUT/A_$r.json
  env $B timeout -k 10 200 python3 bench.py --no-cpu-baseline "$@" > $OUT/B_$r.json
done
