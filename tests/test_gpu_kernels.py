"""Support kernels: column sums (bias / split-K weight gradients) and the split-K Linear
backward against torch fp32 autograd."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda", 0)


@pytest.mark.parametrize("rows,cols", [(262144, 17), (262144, 1), (262144, 64), (256, 24064),
                                       (5000, 376), (3, 5), (4097, 255), (100000, 300)])
def test_sum_rows(dev, rows, cols):
    from tianshou_amd.utils.net import sum_rows
    x = torch.randn(rows, cols, device=dev)
    got = sum_rows(x).double().cpu().numpy()
    want = x.double().sum(0).cpu().numpy()
    np.testing.assert_allclose(got, want, rtol=1e-4, atol=1e-5 * np.sqrt(rows))


@pytest.mark.parametrize("B", [262144, 4096, 1000])
def test_linear_split_k_backward(dev, B):
    from tianshou_amd.utils.net import Linear
    torch.manual_seed(B)
    lin = Linear(376, 64).to(dev)
    ref = torch.nn.Linear(376, 64).to(dev)
    ref.load_state_dict(lin.state_dict())
    x = torch.randn(B, 376, device=dev, requires_grad=True)
    x2 = x.detach().clone().requires_grad_(True)
    g = torch.randn(B, 64, device=dev)
    lin(x).backward(g)
    ref(x2).backward(g)
    for a, b in ((lin.weight.grad, ref.weight.grad), (lin.bias.grad, ref.bias.grad),
                 (x.grad, x2.grad)):
        scale = float(b.abs().max())
        np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-4,
                                   atol=1e-5 * scale)
