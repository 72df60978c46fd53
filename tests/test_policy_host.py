"""Host-side policy logic (no GPU): torch.distributions argument validation around the
policy's distribution construction (tianshou/policy/modelfree/pg.py:133-171 builds
``self.dist_fn(*logits)`` with torch's default validation, so invalid parameters raise
ValueError there)."""
import pytest
import torch


def _gauss(mu, sigma):
    return torch.distributions.Independent(torch.distributions.Normal(mu, sigma), 1)


def test_make_dist_validation_opt_in_and_default_restored():
    from tianshou_amd.policy.pg import make_dist
    default = torch.distributions.Distribution._validate_args
    mu = torch.zeros(3, 2)
    bad = torch.full((3, 2), -1.0)  # negative scale
    with pytest.raises(ValueError):
        make_dist(_gauss, (mu, bad), validate=True)
    d = make_dist(_gauss, (mu, bad))  # the sync-free default: no check, NaN downstream
    assert torch.isnan(d.log_prob(torch.zeros(3, 2))).all()
    assert torch.distributions.Distribution._validate_args == default
    ok = make_dist(_gauss, (mu, torch.ones(3, 2)), validate=True)
    torch.testing.assert_close(ok.log_prob(torch.zeros(3, 2)),
                               _gauss(mu, torch.ones(3, 2)).log_prob(torch.zeros(3, 2)))
    logits = torch.tensor([[0.1, float("nan")]])
    with pytest.raises(ValueError):
        make_dist(lambda p: torch.distributions.Categorical(logits=p), logits, validate=True)
    assert torch.distributions.Distribution._validate_args == default
