"""GradientVerifier (the reference's phantom security/gradient_verification.py, called at
distributed_trainer.py:199-205): host path on CPU gradients, device path on GPU gradients."""
import pytest
import torch

from trustworthy_dl.security.gradient_verification import GradientVerifier


def _grads(gen, scale=1.0, device="cpu"):
    shapes = [(64, 32), (32,), (128, 64)]
    return [(torch.randn(*s, generator=gen) * scale).to(device) for s in shapes]


def _run(device):
    gen = torch.Generator().manual_seed(0)
    gv = GradientVerifier(warmup=10)
    clean = [gv.verify_gradients(_grads(gen, 1.0 + 0.01 * i, device), node_id=3, step=i, ground_truth=False)
             for i in range(30)]
    poisoned = gv.verify_gradients(_grads(gen, 10.0, device), node_id=3, step=30, ground_truth=True)
    after = gv.verify_gradients(_grads(gen, 1.3, device), node_id=3, step=31, ground_truth=False)
    return gv, clean, poisoned, after


def test_gradient_verifier_host_path():
    gv, clean, poisoned, after = _run("cpu")
    assert all(clean[10:]), clean
    assert poisoned is False
    st = gv.statistics()
    assert st["rejected"] >= 1 and st["device_nodes"] == []
    assert gv.node_history(3)[-2]["flagged"] is True


@pytest.mark.gpu
def test_gradient_verifier_device_path():
    gv, clean, poisoned, after = _run("cuda")
    assert all(clean), clean                      # no false positive, warm-up included
    assert poisoned is False                      # x10 gradient rejected
    assert after is True                          # the flagged step did not enter the baseline
    st = gv.statistics()
    assert st["device_nodes"] == [3]
    assert st["total_detections"] == 1 and st["precision"] == 1.0 and st["recall"] == 1.0
    rec = gv.node_history(3)[-2]
    assert rec["path"] == "device" and rec["flagged"] and rec["z"] > 8.0
    # a changed parameter set rebuilds the node's device state
    gen = torch.Generator().manual_seed(1)
    assert gv.verify_gradients([torch.randn(10, generator=gen).cuda()], node_id=3, step=32)
