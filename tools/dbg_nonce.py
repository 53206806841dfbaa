"""Debug: st encode with ZMQG_OPT_NONCE_AUTO -- print wire nonces."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from libzmq_amd import curve as C
for n in (256, 512, 65536):
    P = 1024
    W = P + 33
    ctx = C.CurveContext(0, 1)
    ctx.session_set(0, bytes(range(32)), C.CLIENT_PREFIX, C.SERVER_PREFIX)
    ctx.set_nonce(0, 3)
    t = lambda a, d: torch.from_numpy(np.ascontiguousarray(a).view(d)).cuda()
    sid = t(np.zeros(n, np.uint32), np.int32)
    fl = torch.zeros(n, dtype=torch.uint8, device="cuda")
    ioff = t(np.arange(n, dtype=np.uint64) * P, np.int64)
    lens = t(np.full(n, P, np.uint32), np.int32)
    ooff = t(np.arange(n, dtype=np.uint64) * W, np.int64)
    inp = torch.zeros(n * P, dtype=torch.uint8, device="cuda")
    out = torch.zeros(n * W, dtype=torch.uint8, device="cuda")
    for mode in ("max_len", "none"):
        ctx.set_nonce(0, 3)
        if mode == "max_len":
            ctx.encode_batch(sid, None, fl, ioff, lens, inp, ooff, out, max_len=P, nonce_auto=True)
        else:
            ctx.encode_batch(sid, None, fl, ioff, lens, inp, ooff, out, nonce_auto=True)
        torch.cuda.synchronize()
        w = out.cpu().numpy().reshape(n, W)
        nn = w[:, 8:16].copy().view(">u8").reshape(n)
        print(n, mode, "nonces", nn[:4], nn[250:260], "counter after", ctx.get_nonce(0), "hdr", w[0, :8].tobytes())
