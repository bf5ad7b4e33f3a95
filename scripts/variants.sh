#!/bin/bash
# Build k_solve variants (waves per workgroup, path waves) into lompc_amd/liblompc_amd_<W>_<P>.so
# (diagnostics; the product library keeps the defaults of lompc_plan.hip).
cd "$(dirname "$0")/.." || exit 1
for v in "$@"; do
  W=${v%_*}; P=${v#*_}
  python -c "
import sys; sys.path.insert(0, 'incentive-design-mpc_amd')
from lompc_amd import build
print(build.build(force=True, out='incentive-design-mpc_amd/lompc_amd/liblompc_amd_${W}_${P}.so',
                  defines=('LQ_SOLVE_WAVES=$W', 'LQ_SOLVE_PATHS=$P')))" &
done
wait
