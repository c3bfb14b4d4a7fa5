"""agent.py parity with the reference modules (CPU, fp32): checkpoint loading, forward outputs,
initialisation order, parameter groups."""

import numpy as np
import pytest
import torch

from conftest import golden


@pytest.mark.parametrize("fixture", ["mlp.npz", "mlp196.npz"])
def test_best_model_checkpoint_loads_and_matches_forward(fixture):
    """The reference's best_model.pt (h 192) and a reference GameMLP at the bench's train config
    (h 196, random init): state_dict loads, fp32 forward equals the reference's."""
    import agent
    g = golden(fixture)
    cfg = agent.MLPConfig(hidden_dim=int(g["hidden_dim"]), num_layers=int(g["num_layers"]))
    m = agent.GameMLP(cfg).eval()
    sd = {k[3:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("w::")}
    m.load_state_dict(sd, strict=True)
    with torch.no_grad():
        logits, value = m(torch.from_numpy(g["obs"]))
    np.testing.assert_allclose(logits.numpy(), g["logits"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(value.numpy(), g["value"], rtol=1e-5, atol=1e-5)
    assert agent.param_count(m) == sum(v.size for k, v in ((k, g[k]) for k in g.files if k.startswith("w::")))


def test_init_matches_reference_under_same_seed():
    import agent
    u = golden("update.npz")
    torch.manual_seed(1234)
    m = agent.GameMLP(agent.MLPConfig(hidden_dim=64, num_layers=2, dropout=0.0))
    for k, v in m.state_dict().items():
        assert np.array_equal(v.numpy(), u[f"init::{k}"]), k


@pytest.mark.parametrize("fixture", ["urm.npz", "urm64.npz"])
def test_urm_forward_matches_reference(fixture):
    """agent.GameURM (fp32, CPU) on the reference's weights vs the reference's own forward: the
    small h 32 fixture and the default config (h 64, BASELINE config 5's policy)."""
    import agent
    g = golden(fixture)
    h, L, heads, loops, trunc, k = (int(x) for x in g["config"])
    cfg = agent.GameURMConfig(hidden_dim=h, num_layers=L, num_heads=heads, num_loops=loops,
                              num_truncated_loops=trunc, conv_kernel=k, dropout=0.0,
                              expansion=float(g["expansion"]), rms_norm_eps=float(g["eps"]))
    m = agent.GameURM(cfg).eval()
    m.load_state_dict({kk[3:]: torch.from_numpy(g[kk]) for kk in g.files if kk.startswith("w::")}, strict=True)
    with torch.no_grad():
        logits, value = m(torch.from_numpy(g["obs"]))
    np.testing.assert_allclose(logits.numpy(), g["logits"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(value.numpy(), g["value"], rtol=1e-4, atol=1e-5)


def test_param_groups_and_directions():
    import agent
    m = agent.GameMLP(agent.MLPConfig(hidden_dim=196, num_layers=2))
    o2, o1, v2, v1 = m.get_param_groups(1e-4, 1e-3)
    assert o2["lr"] == 1e-3 and v2["lr"] == 1e-4
    assert [p.shape for p in v2["params"]] == [torch.Size([1, 196])]
    assert [p.shape for p in v1["params"]] == [torch.Size([1])]
    assert all(p.ndim == 2 for p in o2["params"]) and all(p.ndim == 1 for p in o1["params"])
    assert agent.param_count(m) == 88401  # SURVEY.md §8a a9 (h=196, L=2)
    assert [d.value for d in m.directions] == ["up", "down", "left", "right"]
    with pytest.raises(ValueError):
        m(torch.zeros(48))
