# 8-channel throughput: streams per channel, front/back split, AGC chunk length (tuning build)
cd $GRAFT_REPO_ROOT && export LDSP_PKG_DIR=build_tuning
for C in 1024; do for cfg in "2 0" "1 1" "2 1"; do set -- $cfg
  echo "C=$C PER=$1 SPLIT=$2 $(LDSP_AGC_C=$C PER=$1 SPLIT=$2 STEPS=8 timeout -k 10 200 python scripts/channels_run.py 2>/dev/null | tail -1)"
done; done
