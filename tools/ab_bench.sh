#!/bin/bash
# A/B bench: bash tools/ab_bench.sh CFG1 CFG2 ...  (3 rounds, same box)
# A config is words "ENV=val" (environment), "--flag" (extra bench.py argument) and
# "DIR=ab_tree" (the bench of another revision, tools/make_ab_tree.sh).
cd $GRAFT_REPO_ROOT && python -c "import __graft_entry__ as g; g.build()" > /dev/null 2>&1 || exit 3
for i in $(seq ${ROUNDS:-3}); do
  for cfg in "$@"; do
    # a config's words: ENV=val (environment), --flag (bench argument), DIR=path (another tree)
    envs="AB_NONE=1"; args=""; dir=.
    for w in $cfg; do
      if [[ "$w" == DIR=* ]]; then dir=${w#DIR=}
      elif [[ "$w" == --* ]]; then args="$args $w"
      else envs="$envs $w"; fi
    done
    (cd $dir && env $envs timeout -k 10 200 python bench.py --steps ${STEPS:-300} --warmup ${WARMUP:-20} --no-cpu-baseline \
      --no-superbatch --no-kernel-timer --no-finetune $args 2>/dev/null) | tail -1 | \
      python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$cfg', d['ms_per_step'], d['value'])" || exit 1
  done
done
