"""Debug: JPEG member planes on device vs the oracle (GPU box)."""
import ctypes, sys
import numpy as np, torch
sys.path.insert(0, ".")
from s3od_amd._lib import lib, stream
from s3od_amd.data import SynthParams, augment_ws_floats
from oracle import augment_oracle as AO
S = 64
yy, xx = np.mgrid[0:S, 0:S] / S
x = np.stack([xx, yy, 0.5 + 0.3 * np.sin(6 * xx)]).astype(np.float32)
for name, img in (("const", np.full((3, S, S), 0.5, np.float32)), ("grad", x)):
    t = torch.from_numpy(img).cuda()
    ws = torch.zeros(augment_ws_floats(S), device="cuda")
    q = SynthParams.identity(); q.jpeg_quality = 75; q.ws = ws.data_ptr()
    out = torch.empty(3, S, S, device="cuda")
    lib()("s3od_augment_synthetic", t.clone(), ctypes.addressof(q), None, S, out, stream())
    torch.cuda.synchronize()
    MEAN = np.array([0.485, 0.456, 0.406])[:, None, None]; STD = np.array([0.229, 0.224, 0.225])[:, None, None]
    got = out.cpu().numpy() * STD + MEAN
    ref = AO.jpeg(img.astype(np.float64), 75)
    w = ws.cpu().numpy()
    Y = w[3 * S * S: 3 * S * S + S * S].reshape(S, S)
    C = w[4 * S * S: 4 * S * S + 2 * (S // 2) ** 2].reshape(2, S // 2, S // 2)
    print(name, "got-ref mean", np.abs(got - ref).mean(), "got-x", np.abs(got - img).mean(), "ref-x", np.abs(ref - img).mean())
    print(" Y plane sample", Y[0, :8], Y[31, 30:34])
    print(" C planes sample", C[0, 0, :6], C[1, 5, :6])
    print(" got px", got[:, 0, :4].round(4).tolist(), "ref", ref[:, 0, :4].round(4).tolist(), "x", img[:, 0, :4].round(4).tolist())
