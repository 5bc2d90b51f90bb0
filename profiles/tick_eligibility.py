import sys, torch
sys.path.insert(0, 'replication-of-minute-frequency-factor_amd')
from mff import synth
dev = torch.device('cuda:0')
bars, mask = synth.make_panel_device(5000, 2500, dev, config=4)
c = bars[3].double()
k = torch.round(c * 100)
ongrid = ((k * 0.01).float() == bars[3]).all(-1)
rng = k.amax(-1) - k.amin(-1)
print('ongrid', ongrid.float().mean().item())
for t in (256, 512, 1024):
    e = (rng < t).float()
    w = e.view(2500, 1250, 4).amin(-1)  # waves of 4 groups (stocks 4j..4j+3)
    print(t, 'eligible', e.mean().item(), 'wave-all-eligible', w.mean().item())
print('price median', c.median().item(), 'p90', c.flatten()[::997].quantile(0.9).item())
