"""GPU debugging aid: isolates the SigG1 pieces (G2 fixed-base tables, G2 MSM, g~ lines)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "coconut-rust_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import coconut
from conftest import golden, oracle_lib
oc = oracle_lib()
ctx = coconut.Context(0, coconut.GroupMode.SIG_G1)
ks = [5, 123456789, 2**200 + 77]
sc = b"".join(k.to_bytes(48, "big") for k in ks)
for grp, gen, eb in ((1, coconut.G1_GENERATOR, 97), (2, coconut.G2_GENERATOR, 192)):
    got = coconut.fixed_base_mul(ctx, grp, gen, sc)
    ref = ctypes.create_string_buffer(eb * len(ks))
    oc.oc_gen_mul(grp, ctypes.c_size_t(len(ks)), sc, ref)
    print("fixed_base_mul group", grp, "match:", [got[eb*i:eb*(i+1)] == ref.raw[eb*i:eb*(i+1)] for i in range(len(ks))])
d = golden("verify_g1_q6.json")
cr = d["creds"][:4]
ctx.set_params(bytes.fromhex(d["g_tilde"]))
ctx.set_verkey(bytes.fromhex(d["vk"]["X"]), [bytes.fromhex(y) for y in d["vk"]["Y"]])
cat = lambda hs: b"".join(bytes.fromhex(h) for h in hs)
v, gts = coconut.verify_batch(ctx, len(cr), d["q"], cat(c["sigma1"] for c in cr), cat(c["sigma2"] for c in cr),
                              cat(m for c in cr for m in c["msgs"]), want_gt=True)
print("shared-vk verdicts", list(v), "expected", [c["verdict"] for c in cr])
print("gt match", [gts[576*i:576*(i+1)].hex() == c["gt"] for i, c in enumerate(cr)])
X = cat([d["vk"]["X"]] * len(cr)); Y = cat(y for _ in cr for y in d["vk"]["Y"])
v2, gts2 = coconut.verify_batch(ctx, len(cr), d["q"], cat(c["sigma1"] for c in cr), cat(c["sigma2"] for c in cr),
                                cat(m for c in cr for m in c["msgs"]), vk=(X, Y), want_gt=True)
print("per-cred-vk verdicts", list(v2), "gt match", [gts2[576*i:576*(i+1)].hex() == c["gt"] for i, c in enumerate(cr)])
