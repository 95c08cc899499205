import sys, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import __graft_entry__ as g
m = g.package(); m.load_library(); o = g.oracle()
import torch
from conftest import CONFIGS, oracle_phasor, oracle_slicer, product_phasor
for cfg in ["c1_bpsk", "c2_qpsk", "c3_qam16"]:
    name, bps, L, sps = CONFIGS[cfg]
    nsym = 3000
    bits = o.prng_bits(0x5EED0000 + 7, nsym * bps)
    taps = m.rrc_taps(L, sps, 0.35)
    w = o.sample_freq(1, 4)
    x = o.tx_chain(oracle_phasor(o, name), bits, sps, taps, w, 0, flush_syms=(L - 1 + sps - 1) // sps)
    riq, rsym = o.rx_chain(x, w, 0, o.MIX_COMPLEX, taps, sps, L - 1, oracle_slicer(o, name, bps))
    rx = m.DemodulatorRx(m.Carrier(w), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX, slicer=product_phasor(m, name).slicer())
    giq, gsym = rx.process(torch.from_numpy(x).cuda())
    giq = giq.cpu().numpy()
    err = np.abs(giq - riq).max(1)
    bad = np.nonzero(err > 1e-4)[0]
    print(cfg, len(giq), 'bad', len(bad), bad[:20], (bad % 16)[:20] if len(bad) else '', err.max())
    if len(bad): print(giq[bad[:4]], riq[bad[:4]])
