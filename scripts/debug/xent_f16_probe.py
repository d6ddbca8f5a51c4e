"""GPU probe: fused fp16 cross-entropy dW against an fp32 emulation of the same fp16 roundings
(E = fp16(exp(l - c)), xs = fp16(x g / S)), to tell rounding from a kernel error."""
import torch
import torch.nn.functional as F

from nanosandbox_amd import ops

DEV, H16 = "cuda", torch.float16
torch.manual_seed(5)
N, V, C = 1024, 50257, 256
x0 = torch.randn(N, C, device=DEV)
flagged = torch.arange(0, 1000, 10, device=DEV)
x0[flagged] *= 400.0
x0[1::10] *= 6.0
x0 = x0.to(H16)
w0 = torch.randn(V, C, device=DEV) * 0.05
t = torch.randint(0, V, (N,), device=DEV)
t[flagged[::20]] = V - 1
t[3::97] = -1
scale = 1024.0
xs_ = x0.clone().requires_grad_(True)
w = torch.nn.Parameter(w0.clone())
w.main_grad = torch.zeros(V, C, device=DEV)
w.compute = w.detach().to(H16)
loss = ops.lm_head_loss(xs_, w, t)
(loss * scale).backward()
gw = w.main_grad
xr = x0.float()
wr = w0.to(H16).float()
logits = xr @ wr.t()
valid = t >= 0
n_valid = valid.sum().float()
g = scale / n_valid
tt = t.clamp(min=0)
c = logits.gather(1, tt[:, None])
m = logits.max(1, keepdim=True).values
E = torch.exp(logits - c)
over = (E > 65504).any(1, keepdim=True)
E = torch.where(over, torch.exp(logits - m), E)
S = E.sum(1, keepdim=True)
Eh = E.to(H16).float()
xsh = (xr * (g / S)).to(H16).float() * valid[:, None]
dW_em = Eh.t() @ xsh
dW_em.index_add_(0, tt[valid], -(g * xr[valid]))
lr = F.cross_entropy(logits, t, ignore_index=-1) * scale
wq = wr.clone().requires_grad_(True)
(F.cross_entropy(xr @ wq.t(), t, ignore_index=-1) * scale).backward()
ref = wq.grad
print("rows over (fix-up):", int(over.sum()), "of", N)
for name, a in (("kernel", gw), ("emul", dW_em)):
    d = (a - ref).abs()
    i = int(d.argmax())
    print(name, "vs fp32: max abs err", d.max().item(), "at", (i // C, i % C), "rel_err",
          ((a - ref).norm() / ref.norm()).item())
d = (gw - dW_em).abs()
i = int(d.argmax())
print("kernel vs emul: max abs", d.max().item(), "at", (i // C, i % C), "kernel", gw.view(-1)[i].item(), "emul",
      dW_em.view(-1)[i].item(), "ref", ref.view(-1)[i].item())
v, cc = 18922, 185
contrib = (Eh[:, v] * xsh[:, cc])
top = contrib.abs().topk(5)
print("18922,185: kernel", gw[v, cc].item(), "emul", dW_em[v, cc].item(), "ref", ref[v, cc].item())
for k, r in zip(top.values.tolist(), top.indices.tolist()):
    print("  row", r, "contrib", contrib[r].item(), "E", Eh[r, v].item(), "p_exact", (E[r, v] / S[r]).item(),
          "S", S[r].item(), "x", xr[r, cc].item(), "over", bool(over[r]), "t", int(t[r]))
