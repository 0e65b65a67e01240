#!/bin/bash
export TMPDIR=/tmp
bash $GRAFT_REPO_ROOT/tools/gpu_r05_22.sh && bash $GRAFT_REPO_ROOT/tools/gpu_r05_23.sh
