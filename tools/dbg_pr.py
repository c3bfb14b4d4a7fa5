"""Debug: per-layer / head outputs of the fused rollout kernel's first step vs FusedPolicy."""
import sys
import torch
sys.path[:0] = ['.', '2048-ppo_amd', 'tests']
from test_gpu_policy_rollout import _model
from g2048 import _lib as L
from g2048.rollout import FusedPolicy, Rollout
dev = torch.device('cuda', 0)
for h in (196, 64):
    m = _model(dev, h, 7)
    pol = FusedPolicy(m)
    n = 256
    ro = Rollout(n, 2, dev, seed=9)
    ro.reset()
    nt = (h + 15) // 16
    F = 16 * nt
    dbg = torch.zeros(4 * n * F + 5 * n, dtype=torch.float32, device=dev)
    L.policy_rollout(ro.buf, 0, 1, pol.wbf[0], pol.wbf[1:], [x.weight for x in pol.ln], [x.bias for x in pol.ln],
                     pol.head_bf, pol.heads[1], pol.heads[3], ro.seed, ro.env_base, ro.counter, ro.opts, debug=dbg)
    obs = torch.empty(n, 48, dtype=torch.bfloat16, device=dev)
    L.obs_encode(ro.buf.boards[0], obs)
    lg, v = pol(obs)
    hd = dbg[4 * n * F:].view(n, 5)
    for l in range(3):
        got = dbg[l * n * F:(l + 1) * n * F].view(n, F)[:, :h]
        ref = pol.h[l % 2].float() if l == 2 else None
    print(h, 'logits maxdiff', float((hd[:, :4] - lg).abs().max()), 'nbad', int((hd[:, :4] != lg).sum()),
          'value maxdiff', float((hd[:, 4] - v).abs().max()), 'nbad', int((hd[:, 4] != v).sum()))
    # sampler on identical logits: per-step kernel vs the fused records
    act = torch.zeros(n, dtype=torch.uint8, device=dev)
    lp = torch.zeros(n, 4, device=dev)
    en = torch.zeros(n, device=dev)
    L.sample_actions(hd[:, :4].contiguous(), ro.buf.flags[0], act, lp, en,
                     L.make_rng(L.RNG_PHILOX, ro.seed, 0, ro.env_base, counter_dev=ro.counter))
    print(h, 'sampler on kernel logits: actions equal', bool(torch.equal(act, ro.buf.actions[0])),
          'logp bitwise', bool(torch.equal(lp.view(torch.int32), ro.buf.logp[0].view(torch.int32))),
          'entropy bitwise', bool(torch.equal(en.view(torch.int32), ro.buf.entropy[0].view(torch.int32))),
          'logp maxdiff', float(torch.nan_to_num((lp - ro.buf.logp[0]).abs(), nan=0).max()))
