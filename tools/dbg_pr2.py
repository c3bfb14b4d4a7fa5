"""Debug: the bitwise test configuration, printing the mismatching records and checking run-to-run
determinism of both paths."""
import sys
import torch
sys.path[:0] = ['.', '2048-ppo_amd', 'tests']
from test_gpu_policy_rollout import _model, _run
dev = torch.device('cuda', 0)
m = _model(dev, 196, 196 + 4099)
ref = _run(dev, m, 4099, 24, fused=False)
ref2 = _run(dev, m, 4099, 24, fused=False)
got = _run(dev, m, 4099, 24, fused=True)
got2 = _run(dev, m, 4099, 24, fused=True)
for name, a, b in (("ref-vs-ref2", ref, ref2), ("got-vs-got2", got, got2), ("ref-vs-got", ref, got)):
    for k in ("value", "logp", "entropy", "actions", "boards"):
        x, y = a[k], b[k]
        if x.dtype.is_floating_point:
            xi, yi = x.view(torch.int32), y.view(torch.int32)
        else:
            xi, yi = x, y
        bad = (xi != yi).reshape(x.shape[0], x.shape[1], -1).any(-1)
        print(name, k, int(bad.sum()))
        if k in ("value", "logp") and bad.any() and name == "ref-vs-got":
            for t, i in torch.nonzero(bad)[:4].tolist():
                print('    t', t, 'i', i, 'ref', x[t, i].tolist(), 'got', y[t, i].tolist(),
                      'board', ref["boards"][t, i].tolist(), 'flags', int(ref["flags"][t, i]))
