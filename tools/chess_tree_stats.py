import sys, numpy as np, torch
sys.path.insert(0, '/root/repo')
import oracle
from zeroclone_amd import _native
G, S, B = 64, 400, 32
eng = _native.NativeEngine(max_games=G, max_sims=S, max_batch=B)
rs = np.random.default_rng(5)
roots = []
for i in range(G):
    st = oracle.chess_init()
    for _ in range(int(rs.integers(0, 24)) if i % 2 else 0):
        ms = oracle.chess_moves(st)
        if not ms: break
        nxt = oracle.chess_play(st, ms[int(rs.integers(0, len(ms)))])
        if oracle.chess_win(nxt) or oracle.chess_draw(nxt) or not oracle.chess_moves(nxt): break
        st = nxt
    r = np.zeros(1, _native.CHESS_STATE_DTYPE)
    r["board"][0] = np.frombuffer(bytes(st.board), np.uint8)
    r["turn"], r["fifty"], r["castle"] = st.turn, st.fifty, st.castle
    roots.append(r)
roots = torch.from_numpy(np.concatenate(roots).view(np.uint8).reshape(G, 72).copy()).cuda()
mv = torch.zeros(G, dtype=torch.int16, device="cuda"); na = torch.zeros((G, 256), dtype=torch.int32, device="cuda")
st = torch.zeros((G, 8), dtype=torch.int64, device="cuda")
eng.seed(0, list(range(G)))
eng.chess_search_async(0, G, roots.data_ptr(), S, 1.4, B, 1, 3.0, mv.data_ptr(), na.data_ptr(), st.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
tot = exp = term = 0
for g in range(G):
    t = eng.debug_chess_tree(g)
    n = t["nodes"]
    tot += len(n); exp += int((n["nu"] < n["nmoves"]).sum()); term += int((n["nmoves"] == 0).sum())
print("nodes", tot, "expanded>=1 child", exp, "terminal", term, "never expanded frac", 1 - exp / tot)
