"""Debug: layer-0 statistics on specific boards (found mismatching in the bitwise test)."""
import sys
import numpy as np
import torch
sys.path[:0] = ['.', '2048-ppo_amd', 'tests']
from test_gpu_policy_rollout import _model
from g2048 import _lib as L
from g2048.rollout import FusedPolicy, Rollout
dev = torch.device('cuda', 0)
h = 196
m = _model(dev, h, 196 + 4099)
pol = FusedPolicy(m)
n = 256
ro = Rollout(n, 2, dev, seed=9)
ro.reset()
bad_boards = [[3, 2, 0, 1, 2, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0], [3, 2, 2, 0, 3, 1, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0]]
for k, bb in enumerate(bad_boards):
    ro.buf.boards[0][k] = torch.tensor(bb, dtype=torch.int8, device=dev)
L.legal_mask(ro.buf.boards[0], ro.buf.flags[0])
nt = (h + 15) // 16
F = 16 * nt
dbg = torch.zeros(4 * n * F + 5 * n, dtype=torch.float32, device=dev)
L.policy_rollout(ro.buf, 0, 1, pol.wbf[0], pol.wbf[1:], [x.weight for x in pol.ln], [x.bias for x in pol.ln],
                 pol.head_bf, pol.heads[1], pol.heads[3], ro.seed, ro.env_base, ro.counter, ro.opts, debug=dbg)
obs = torch.empty(n, 48, dtype=torch.bfloat16, device=dev)
L.obs_encode(ro.buf.boards[0], obs)
y = torch.empty(n, h, dtype=torch.bfloat16, device=dev)
G = torch.empty(n, h, dtype=torch.bfloat16, device=dev)
mean = torch.empty(n, device=dev)
rstd = torch.empty(n, device=dev)
L.mlp_fwd(obs, pol.wbf[0], pol.ln[0].weight, pol.ln[0].bias, False, G, y, mean, rstd, None)
st = dbg[3 * n * F:4 * n * F].view(n, F)[:, :3]
got = dbg[:n * F].view(n, F)[:, :h]
f32 = np.float32
for i in range(2):
    s_, v_, r_ = (float(x) for x in st[i])
    print('board', i, 'kernel sum', s_, 'var', v_, 'rstd', r_, '| mlp_fwd mean', float(mean[i]), 'rstd', float(rstd[i]),
          '| sum*inv_n', float(f32(s_) * (f32(1) / f32(196))))
    bad = torch.nonzero(got[i] != y[i].float())[:, 0].tolist()
    for j in bad:
        gj = f32(G[i, j].float().item())
        gam, bet = f32(pol.ln[0].weight[j].item()), f32(pol.ln[0].bias[j].item())
        inv = f32(1) / f32(196)
        dv_fma = f32(np.float64(gj) - np.float64(f32(s_)) * np.float64(inv))
        dv_sub = f32(gj - f32(f32(s_) * inv))
        for nm, dv in (("fma", dv_fma), ("sub", dv_sub)):
            t = f32(dv * f32(r_))
            yy = f32(np.float64(gam) * np.float64(t) + np.float64(bet))
            print('   feature', j, nm, 'dv', float(dv), 'y', float(yy), 'relu', max(float(yy), 0.0))
        print('   got', float(got[i, j]), 'ref', float(y[i, j].float()), 'G', float(gj))
print('--- numpy emulation of the LN statistics (lane-group sums, xor-16 / xor-32) ---')
for i in range(2):
    gv = G[i].float().cpu().numpy().astype(np.float32)
    gpad = np.zeros(16 * nt, np.float32)
    gpad[:h] = gv
    S = []
    for gg in range(4):
        s_ = f32(0)
        for nn in range(nt):
            for r in range(4):
                fidx = 16 * nn + 4 * gg + r
                s_ = f32(s_ + (gpad[fidx] if fidx < h else f32(0)))
        S.append(s_)
    tot = f32(f32(S[0] + S[1]) + f32(S[2] + S[3]))
    inv = f32(1) / f32(196)
    V = []
    for gg in range(4):
        v_ = f32(0)
        for nn in range(nt):
            for r in range(4):
                fidx = 16 * nn + 4 * gg + r
                dv = f32(np.float64(gpad[fidx]) - np.float64(tot) * np.float64(inv)) if fidx < h else f32(0)
                v_ = f32(np.float64(dv) * np.float64(dv) + np.float64(v_))
        V.append(v_)
    var = f32(f32(V[0] + V[1]) + f32(V[2] + V[3]))
    x = f32(np.float64(var) * np.float64(inv) + np.float64(f32(1e-5)))
    r = f32(np.float64(1) / np.float64(f32(np.sqrt(np.float64(x)))))
    print('board', i, 'sum', float(tot), 'var', float(var), 'rstd', float(r))
