set -u
export ZD_EXP_KMASK=7
UMIB=1024 REPS=10 bash scripts/bench_variants.sh base e_nostore e_noload e_noboth
