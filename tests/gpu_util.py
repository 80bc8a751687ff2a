import torch

BF16 = torch.bfloat16


def to_dev(t):
    return t.to("cuda")


def err(a, b):
    """(max abs error, relative L2 error) of a bf16 result vs a reference."""
    a, b = a.float().cpu(), b.float().cpu()
    d = (a - b)
    return d.abs().max().item(), (d.norm() / (b.norm() + 1e-30)).item()
