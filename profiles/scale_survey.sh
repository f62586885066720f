#!/bin/bash
# Every method (-m 0 = 1..20) at a larger shape through the CLI on one MI355X: looks for
# schedules whose host planning or device execution falls off a cliff.
# usage: profiles/scale_survey.sh <outdir> [procs] [aggs] [d] [c]
out=${1:-gpurun_out/survey}; mkdir -p $out; cd $out
P=${2:-4096}; A=${3:-64}; D=${4:-2048}; C=${5:-8}
bin=$GRAFT_REPO_ROOT/mpi-asynchronous-communication-test_amd/bin/test
t0=$(date +%s.%N)
timeout -k 10 ${SURVEY_TIMEOUT:-500} $bin --procs $P -a $A -d $D -c $C -m 0 -i 1 -p 64 > survey_P${P}_A${A}_d${D}_c${C}.txt 2> err.txt || { echo failed; exit 1; }
python3 -c "import sys; print('wall %.1f s' % (float(sys.argv[2]) - float(sys.argv[1])))" $t0 $(date +%s.%N) >> survey_P${P}_A${A}_d${D}_c${C}.txt
echo done
