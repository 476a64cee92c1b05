"""Diagnostic: per-phase cycle split of the split-client local-training kernel (stamp build).
Run with FEDSIM_LIB=<pkg>/libfedsim_stamps.so on the GPU box."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fedamw_amd
from fedamw_amd import engine, rng, data
dev = torch.device('cuda')
N = int(sys.argv[1]) if len(sys.argv) > 1 else 100
d = data.federated(N, 512, 2048, 10, 1000, device=dev)
feats = engine.Features(d['X_train'], d['y_train'], 2048, dev)
tr = engine.LocalTrainer(feats, 10, 32, 2, split=(int(sys.argv[2]) if len(sys.argv) > 2 else None))
ws_extra = N * tr.G * 16 * 8
tr.ws = torch.zeros(tr.ws.numel() + ws_extra, dtype=torch.uint8, device=dev)
torch.manual_seed(0)
tr.upload_perms(rng.draw_pass_seeds(N * 2))
W0 = torch.zeros(10, feats.ld, device=dev)
for _ in range(3):
    tr.run(W0, 0.5, False, 0, False, 0, False)
torch.cuda.synchronize()
st = tr.ws[-ws_extra:].view(torch.int64).view(-1, 16).cpu().numpy().astype(np.float64)
st = st[st[:, 15] > 0]
steps = st[:, 15]
names = (["fwd", "B3", "publish", "img", "doL", "B1", "softmax+B2", "bwd", "-", "check"] if os.environ.get("PAIR") else
         ["fwd", "S1", "sum+publish", "poll+sum", "img+next", "S2", "softmax+S3", "bwd"])
per = st[:, :len(names)] / steps[:, None]
print('G', tr.G, 'blocks', len(st), 'steps', steps[0])
for k, nm in enumerate(names):
    print('%-12s mean %8.0f  min %8.0f  max %8.0f cycles/step' % (nm, per[:, k].mean(), per[:, k].min(), per[:, k].max()))
print('total       mean %8.0f cycles/step' % per.sum(1).mean())
print('re-polls per step (wave 0): mean %.3f max %.3f' % ((st[:, 11] / steps).mean(), (st[:, 11] / steps).max()))
