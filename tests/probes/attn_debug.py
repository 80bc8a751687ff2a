import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import kernels as K
from oracle import wan_oracle as O
BF = torch.bfloat16
def run(q, k, v, H=1):
    B, S, D = q.shape
    out = torch.empty(B * S, D, dtype=BF, device="cuda")
    K.attention(q.cuda().view(B*S, D), k.cuda().view(B*k.shape[1], D), v.cuda().view(B*k.shape[1], D), out, H, B)
    torch.cuda.synchronize()
    return out.view(B, S, D).cpu()
g = torch.Generator().manual_seed(0)
S = 256
v = torch.randn(1, S, 128, generator=g).to(BF)
k = torch.randn(1, S, 128, generator=g).to(BF)
# (a) q = 0: uniform softmax
q = torch.zeros(1, S, 128).to(BF)
o = run(q, k, v); ref = O.attention(q, k, v, 1)
print("a uniform: maxerr", (o.float()-ref.float()).abs().max().item())
print(" row0 got", o[0,0,:8].float().tolist()); print(" row0 ref", ref[0,0,:8].float().tolist())
# (b) v = key index in column 0 (and j in col j), q = 0 -> mean
v2 = torch.zeros(1, S, 128); v2[0, :, 0] = torch.arange(S) / S; v2[0, 5, 3] = 1.0
v2 = v2.to(BF)
o = run(q, k, v2); ref = O.attention(q, k, v2, 1)
print("b: got col0/3", o[0, 0, 0].item(), o[0, 0, 3].item(), " ref", ref[0,0,0].item(), ref[0,0,3].item())
print(" nonzero cols of row0:", torch.nonzero(o[0,0].float().abs() > 1e-4).flatten().tolist())
# (c) sharp attention: q_i = 8*e_?; keys one-hot -> query i attends key i
q3 = torch.zeros(1, S, 128); k3 = torch.zeros(1, S, 128)
for i in range(S):
    q3[0, i, i % 128] = 30.0; k3[0, i, i % 128] = 1.0
v3 = torch.zeros(1, S, 128); v3[0, :, 0] = torch.arange(S).float()
o = run(q3.to(BF), k3.to(BF), v3.to(BF))
ref = O.attention(q3.to(BF), k3.to(BF), v3.to(BF), 1)
print("c: got", o[0, :12, 0].float().tolist()); print("   ref", ref[0, :12, 0].float().tolist())
print("c rows 32..40 got", o[0, 32:40, 0].float().tolist())
# (d) random full
qr = torch.randn(1, S, 128, generator=g).to(BF)
o = run(qr, k, v); ref = O.attention(qr, k, v, 1)
print("d random maxerr", (o.float()-ref.float()).abs().max().item())
