# kernel breakdown of the sorted embedding backward at the GPT-2 training shape
scripts/gpu_session.sh \
 "prof_emb|200|cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_emb -o run -- python3 scripts/emb_bwd_ab.py --B 120 --T 1024 --rounds 3"
