cd $GRAFT_REPO_ROOT && python -c "import __graft_entry__ as g; g.build()" > /dev/null 2>&1 || exit 3
for i in 1 2 3; do
  for e in 0 1; do
    SCGIB_EGO_FIRST=$e timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-superbatch --no-kernel-timer 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('ego_first=$e', d['ms_per_step'], d['value'])" || exit 1
  done
done
