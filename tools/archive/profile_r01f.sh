# r01f profiles: headline RS(10,4) (bench defaults) and BASELINE config 5
# RS(64,16) 64 KiB shards (bit-sliced encode + split reconstruct).
set -o pipefail
PROF_TAG=r01f bash tools/profile.sh || exit 1
PROF_TAG=r01f_cfg5 PROF_ARGS="--k 64 --n 80 --shard 65536 --stripes 16384 --emax 16 --pattern-pool 256" bash tools/profile.sh || exit 1
