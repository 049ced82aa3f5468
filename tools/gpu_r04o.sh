set -o pipefail
STAMP_ARGS="--utt" bash tools/stamps.sh r04o_ibm 0 && \
STAMP_ARGS="--utt --mask ipd --batch 1024" bash tools/stamps.sh r04o_ipd 0
