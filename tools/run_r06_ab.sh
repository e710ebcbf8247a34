# Same-process A/Bs of the shipped SYRK forms on one GPU box (via gpurun), K compared bit for bit:
# the f64 residue SYRK (hook crt: 1 = shipped k_syrk_i8w, 2 = without its schedule settings,
# 0 = k_syrk_i8r), the per-block moduli (hook crt_block) and the fp16x2 SYRK (hook h2).
#   bash tools/run_r06_ab.sh <tag>   -> gpurun_out/<tag>/
set -e
OUT=gpurun_out/${1:-r06ab}
mkdir -p $OUT
timeout -k 10 300 python -u tools/ab_crt.py --dtype f64 --n 50000 --m 62500 --rounds 3 --forms 1,2,0 > $OUT/ab_crt_n50k.jsonl 2> $OUT/ab_crt_n50k.err
timeout -k 10 300 python -u tools/ab_crt.py --dtype f64 --hook crt_block --n 50000 --m 62500 --rounds 2 --forms 1,0 > $OUT/ab_crt_block_n50k.jsonl 2> $OUT/ab_crt_block_n50k.err
timeout -k 10 300 python -u tools/ab_crt.py --dtype f32 --n 50000 --m 62500 --rounds 3 --forms 1,0 > $OUT/ab_h2_n50k.jsonl 2> $OUT/ab_h2_n50k.err
echo ab-done
