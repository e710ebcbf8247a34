# A/B of SYRK variants in one process (ubench build): tools/run_syrk_ab.sh <tag> <variants> [n m]
set -e
TAG=$1; V=$2; NN=${3:-50000}; MM=${4:-10000}
mkdir -p gpurun_out/$TAG
export SNPMI_LIB=tools/libsnpmi_ubench.so
timeout -k 10 300 python tools/ubench.py syrk --n $NN --m $MM --variants $V --rounds 5 --noassert 1 >> gpurun_out/$TAG/ubench_syrk.jsonl 2>> gpurun_out/$TAG/ubench.err
echo ok
