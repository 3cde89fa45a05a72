#!/bin/bash
# Reproducer of the r05m class-2 wrong-code kernel (profiles/README.md r06s-u), on the
# build host: a checkout of the source in which it was found, its d3q27_tePSM_per_NEBB
# library built without the class-2 register floor (c2w0) and with one backend stage
# switched per variant; then on a GPU box: TAG=... scripts/gpu_session.sh c2old
set -e
R=$(cd "$(dirname "$0")/.." && pwd); cd $R
[ -d _wt_c2 ] || git worktree add -f _wt_c2 2088283
python - <<'PY'
import re
new = open("tclb_amd/build.py").read()
p = "_wt_c2/tclb_amd/build.py"
s = open(p).read()
if '"c2w0_nohrp"' not in s:
    block = new[new.index('    "c2w0_noagpr"'):new.index('    "cw2"')]
    k = s.index('    "cw2"')
    open(p, "w").write(s[:k] + block + s[k:])
PY
cd _wt_c2
python -c "from tclb_amd import build as B; B.build_tools(); B.build_device_runtime(); B.build_model('d3q27_tePSM_per_NEBB', kinds=('cpu',))"
for v in ${C2VARIANTS:-c2w0 c2w0_noagpr c2w0_nomisched c2w0_nopostra c2w0_nohrp c2w0_o1}; do
  python -c "from tclb_amd import build as B; B.build_model('d3q27_tePSM_per_NEBB', kinds=('hip',), variant='$v')" &
done
wait
