"""Debug: inject a fifty-move-next position into chess pools and print device vs oracle rows."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import oracle
from zeroclone_amd import _native
from zeroclone_amd.selfplay import ChessSelfPlay
from zeroclone_amd.engine.games.chess import chess_backend as cb
import test_gpu_pools as T

G = 16
crude = ChessSelfPlay(G, 32, batch_size=8, seed=3)
crude.run(3)
crude.take()
for mode in ("step_crude", "valuenet"):
    if mode == "valuenet":
        from zeroclone_amd.nets import ValueNetwork, for_inference
        torch.manual_seed(0)
        model = for_inference(ValueNetwork(128, 2).eval(), "cuda", torch.float16)
        pool = ChessSelfPlay(G, 32, batch_size=8, seed=4, net=model, policy=_native.ZC_POLICY_RANDOM, freedom=0.0)
        pool.adopt(crude)
    else:
        pool = crude
    T.inject_fifty(pool, [5])
    torch.cuda.synchronize()
    r0 = pool.roots.cpu().numpy()[5].copy()
    print(mode, "root row", r0[:67].tolist(), "hlen", pool.hlen.cpu().numpy()[5].tolist())
    res = pool.step().cpu().numpy()
    post = pool.post.cpu().numpy()[5]
    mv = int(pool.moves.cpu().numpy()[5]) & 0xFFFF
    print(mode, "move", _native.unpack_chess_move(mv), "res", int(res[5]))
    print(mode, "post row", post[:67].tolist())
    s = T.ostate(r0, np.zeros((2, 4), np.int16), np.zeros(2, np.int32))
    (fr, fc, tr, tc), v = _native.unpack_chess_move(mv)
    s2 = oracle.chess_play(s, (fr, fc, tr, tc, v))
    print(mode, "oracle post", list(s2.board) == list(post[:64]), s2.turn, s2.fifty, s2.castle, "judge", T.judge(s2))
    print(mode, "err", pool.err.cpu().tolist())
