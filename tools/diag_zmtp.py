import sys, zlib, numpy as np, torch
sys.path.insert(0, '.')
from tests import test_zmtp as T
from oracle import oracle as O
from oracle import zmtp_oracle as Z
from libzmq_amd import curve as C
case = "clean"
dev = torch.device("cuda", 0)
for rep in range(3):
    rng = np.random.default_rng(zlib.crc32(case.encode()))
    precom = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    stream, max_msg, max_frames = T._stream_case(rng, case, precom)
    ref = Z.parse(stream, max_msg, None)
    fr = ref["frames"]; nf = len(fr)
    f_len = np.array([f[2] for f in fr], np.uint32)
    ctx = C.CurveContext(0, 1)
    ctx.session_set(0, precom, C.SERVER_PREFIX, C.CLIENT_PREFIX, False, 2)
    cap = 1000
    inp = np.frombuffer(stream, np.uint8)
    d_in = torch.from_numpy(inp.copy()).to(dev)
    d_foff = torch.zeros(cap, dtype=torch.int64, device=dev)
    d_flen = torch.zeros(cap, dtype=torch.int32, device=dev)
    d_poff = torch.zeros(cap, dtype=torch.int64, device=dev)
    d_out = torch.full((len(stream) + 1,), 0x77, dtype=torch.uint8, device=dev)
    d_fl = torch.zeros(cap, dtype=torch.uint8, device=dev)
    d_st = torch.full((cap,), -1, dtype=torch.int32, device=dev)
    r = ctx.decode_zmtp(0, d_in, len(stream), max_msg, max_frames, d_foff, d_flen, d_poff, d_out, d_fl, d_st)
    st = d_st[:nf].cpu().numpy()
    bad = np.nonzero(st != 0)[0]
    print("rep", rep, "frames", nf, r, "bad", len(bad), "idx", bad[:20].tolist(), "len", f_len[bad[:20]].tolist(), "st", [hex(x) for x in st[bad[:5]]], flush=True)
    print("   peer after", ctx.get_peer_nonce(0), "lens of frames", np.unique(f_len).tolist()[:10])
