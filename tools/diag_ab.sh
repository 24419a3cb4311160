# per-variant rollout statistics and phase cycles: bash tools/diag_ab.sh ab/libX.so ...
for l in "$@"; do
  echo "== $l"
  ZC_LIB=$GRAFT_REPO_ROOT/$l timeout -k 10 120 python -c "
import sys; sys.path.insert(0,'.')
import torch, numpy as np
from zeroclone_amd import _native
eng=_native.NativeEngine(max_games=4096,max_sims=800,max_batch=32)
roots=np.zeros(4096,_native.C4_STATE_DTYPE)
eng.seed(0,list(range(4096)))
mv,na,st=eng.c4_search(roots,800,1.4,32)
print('blocks/leaf', st['rollout_blocks'].sum()/st['leaves'].sum(), 'plies/leaf', st['rollout_plies'].sum()/st['leaves'].sum(), 'words/leaf', st['rng_words'].sum()/st['leaves'].sum())
eng.phase_cycles(True)
eng.seed(0,list(range(4096)))
eng.c4_search(roots,800,1.4,32)
ph=eng.phase_cycles(False)
print({k: round(v/4096/800,1) for k,v in ph.items()})
" || exit 1
done
