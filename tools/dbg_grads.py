import sys, torch
sys.path.insert(0, '.')
import cosnet_amd as C
from cosnet_amd import loss as L
from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs
from oracle.model_ref import RefModel, loss_bce_l1
dev = torch.device('cuda:0')
torch.set_num_threads(16)
m = C.build_model(torch.float32)
sd = recipe_state_dict(m.state_dict())
m.load_state_dict(sd)
m = m.to(dev).train()
ra, rb, da, db, ga, gb = synthetic_inputs(2, 65, 65, seed=7)
x1, x2, labels = m(ra.to(dev), rb.to(dev), da.to(dev), db.to(dev))
loss = L.bce_l1(x1, ga.to(dev)) + L.bce_l1(x2, gb.to(dev))
loss.backward()
torch.cuda.synchronize()
for dt in (torch.float64, torch.float32):
    ref = RefModel(sd, dtype=dt)
    r1, r2, rl = ref.forward(*(t.to(dt) for t in (ra, rb, da, db)))
    rloss = loss_bce_l1(r1, ga.to(dt)) + loss_bce_l1(r2, gb.to(dt))
    rloss.backward()
    if dt == torch.float64:
        ref64 = ref
    else:
        ref32 = ref
rows = []
for k, p in m.named_parameters():
    if p.grad is None:
        continue
    g = p.grad.double().cpu()
    r = ref64.p[k].grad
    r32 = ref32.p[k].grad.double()
    if r is None:
        print('no ref grad', k); continue
    n = r.norm().item()
    rows.append(((g - r).norm().item() / max(n, 1e-30), (r32 - r).norm().item() / max(n, 1e-30), n, k))
rows.sort(reverse=True)
for e, f, n, k in rows[:25]:
    print('%.3e  floor %.3e  norm %.3e  %s' % (e, f, n, k))
print('x1 err', (x1.double().cpu() - r1.double().detach()).abs().max().item())
