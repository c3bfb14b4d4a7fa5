"""Debug: per-layer / head outputs of the fused rollout kernel's first step vs FusedPolicy."""
import sys
import torch
sys.path[:0] = ['.', '2048-ppo_amd', 'tests']
from test_gpu_policy_rollout import _model
from g2048 import _lib as L
from g2048.rollout import FusedPolicy, Rollout
dev = torch.device('cuda', 0)
for h, seed in ((196, 196 + 4099), (64, 64 + 777)):
    m = _model(dev, h, seed)
    pol = FusedPolicy(m)
    n = 65536
    ro = Rollout(n, 2, dev, seed=9)
    ro.reset()
    nt = (h + 15) // 16
    F = 16 * nt
    dbg = torch.zeros(4 * n * F + 5 * n, dtype=torch.float32, device=dev)
    L.policy_rollout(ro.buf, 0, 1, pol.wbf[0], pol.wbf[1:], [x.weight for x in pol.ln], [x.bias for x in pol.ln],
                     pol.head_bf, pol.heads[1], pol.heads[3], ro.seed, ro.env_base, ro.counter, ro.opts, debug=dbg)
    obs = torch.empty(n, 48, dtype=torch.bfloat16, device=dev)
    L.obs_encode(ro.buf.boards[0], obs)
    x = obs
    for l in range(3):
        y = torch.empty(n, h, dtype=torch.bfloat16, device=dev)
        G = torch.empty(n, h, dtype=torch.bfloat16, device=dev)
        mean = torch.empty(n, device=dev)
        rstd = torch.empty(n, device=dev)
        L.mlp_fwd(x, pol.wbf[l], pol.ln[l].weight, pol.ln[l].bias, l > 0, G, y, mean, rstd, None)
        got = dbg[l * n * F:(l + 1) * n * F].view(n, F)[:, :h]
        bad = (got != y.float()).any(1)
        print(h, 'layer', l, 'boards with any mismatch', int(bad.sum()), 'elements', int((got != y.float()).sum()))
        if bad.any():
            i = int(torch.nonzero(bad)[0])
            j = torch.nonzero(got[i] != y[i].float())[:4, 0].tolist()
            print('   board', i, 'features', j, 'got', got[i, j].tolist(), 'ref', y[i, j].float().tolist(),
                  'mean', float(mean[i]), 'rstd', float(rstd[i]))
        x = y
    lg, v = pol(obs)
    hd = dbg[4 * n * F:].view(n, 5)
    badl = (hd[:, :4] != lg).any(1) | (hd[:, 4] != v)
    print(h, 'heads: boards with mismatch', int(badl.sum()))
    if badl.any():
        i = int(torch.nonzero(badl)[0])
        print('   board', i, 'got', hd[i].tolist(), 'ref', lg[i].tolist(), float(v[i]))
    # sampler records at step 0 vs the per-step sampler on the same logits
    act = torch.zeros(n, dtype=torch.uint8, device=dev)
    lp = torch.zeros(n, 4, device=dev)
    en = torch.zeros(n, device=dev)
    L.sample_actions(lg.contiguous(), ro.buf.flags[0], act, lp, en,
                     L.make_rng(L.RNG_PHILOX, ro.seed, 0, ro.env_base, counter_dev=ro.counter))
    bl = (lp.view(torch.int32) != ro.buf.logp[0].view(torch.int32)).any(1)
    print(h, 'sampler: action mismatches', int((act != ro.buf.actions[0]).sum()), 'logp rows', int(bl.sum()),
          'entropy', int((en.view(torch.int32) != ro.buf.entropy[0].view(torch.int32)).sum()))
    if bl.any():
        i = int(torch.nonzero(bl)[0])
        print('   row', i, 'logits', lg[i].tolist(), 'legal', int(ro.buf.flags[0][i]), 'got', ro.buf.logp[0][i].tolist(), 'ref', lp[i].tolist())
