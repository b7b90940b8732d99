"""SASRec float32-vs-float64 gradient conditioning: the
reference step (oracle.sasrec_forward_user, model/sasrec.py:385-435) at the
C4 shape (B 2048, lengths U[5, 50], d 128, h 2, L 2) with random parameters,
run on the host in float64 and float32: relative max error of every
gradient, then again with the ReLU masks of the blocks fixed from the
float64 forward.  Host only (no GPU); output: profiles/round4_sasrec_relu_conditioning.txt."""
import sys

import torch
sys.path.insert(0,'.')
from oracle import lightgcn_oracle as O
F=torch.nn.functional
torch.manual_seed(0)
B,T,d,L,h=2048,50,128,2,2
M=100000
base={"W":torch.randn(M,d)*0.1}
for i in range(L):
    base[f"in_w{i}"]=torch.randn(3*d,d)*d**-0.5; base[f"in_b{i}"]=torch.zeros(3*d)
    base[f"out_w{i}"]=torch.randn(d,d)*d**-0.5; base[f"out_b{i}"]=torch.zeros(d)
    base[f"ln1_w{i}"]=torch.ones(d); base[f"ln1_b{i}"]=torch.zeros(d)
    base[f"ln2_w{i}"]=torch.ones(d); base[f"ln2_b{i}"]=torch.zeros(d)
    base[f"ffn_w{i}"]=torch.randn(d,d)*d**-0.5; base[f"ffn_b{i}"]=torch.zeros(d)
length=torch.randint(5,51,(B,)); items=torch.randint(0,M,(B,T)); pos=torch.randint(0,M,(B,)); neg=torch.randint(0,M,(B,))
def run(dt):
    P={k:v.to(dt).clone().requires_grad_(True) for k,v in base.items()}
    mask=(torch.arange(T)[None,:]<length[:,None]).to(dt)
    x=P["W"][items]*mask[...,None]
    u=O.sasrec_forward_user(x,length,P,h,L)
    loss=F.softplus((u*P["W"][neg]).sum(1)-(u*P["W"][pos]).sum(1)).mean()
    loss.backward()
    return {k:v.grad.double() for k,v in P.items()}
g64=run(torch.float64); g32=run(torch.float32)
for k in g64:
    b=g64[k]; a=g32[k]
    print(k, float((a-b).abs().max()/b.abs().max()))
print("--- same with the pre-activation mask fixed from float64")
_relu=torch.Tensor.relu
masks=[]
def rec(self):
    masks.append((self.detach()>0)); return _relu(self)
torch.Tensor.relu=rec
run(torch.float64)
it=iter(masks)
torch.Tensor.relu=lambda self: self*next(it).to(self.dtype)
g32=run(torch.float32)
for k in g64:
    b=g64[k]; a=g32[k]
    print(k, float((a-b).abs().max()/b.abs().max()))
