bash scripts/iter.sh && K=1 VARIANTS="abl_W1SKIP" bash scripts/ablate.sh
