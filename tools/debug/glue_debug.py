import sys
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
sys.path.insert(0, "tests/golden")
import torch
import make_golden_glue as MG
from onetrainer_amd import kernels as K
from onetrainer_amd.model.StableDiffusionXLModel import NoiseScheduler
from oracle import diffusion as OD

dev = torch.device("cuda:0")
FIX = torch.load("tests/golden/glue_fixtures.pt", weights_only=True)
for key in ["sdxl_epsilon_0", "sdxl_epsilon_7"]:
    f = FIX[key]
    b = MG.sdxl_batch()
    lat = b["latent_image"].permute(0, 2, 3, 1).contiguous().to(dev)
    noise = f["noise"].permute(0, 2, 3, 1).contiguous().to(dev)
    t = f["timestep"].to(dev, torch.int32)
    ns = NoiseScheduler(dev)
    unet_in, target, scaled = K.ddpm_prologue(lat, noise, t, ns.coeffs, 0.13025, 0)
    ours = unet_in[..., :4].permute(0, 3, 1, 2).cpu()
    ref = f["sample"]
    x0 = b["latent_image"] * 0.13025
    xt = OD.add_noise_ddpm(x0, f["noise"], f["timestep"].long(), OD.scaled_linear_betas())
    mism = (ours != ref)
    print(key, "mismatch", mism.sum().item(), "oracle==ref", torch.equal(xt.bfloat16(), ref),
          "scaled==x0", torch.equal(scaled.permute(0, 3, 1, 2).cpu(), x0))
    if mism.any():
        idx = mism.nonzero()[:5]
        for i in idx:
            i = tuple(i.tolist())
            print(i, ours[i].item(), ref[i].item(), xt[i].item())
    # torch on GPU restatement
    co = ns.coeffs
    a = co[1][t.long()].view(2, 1, 1, 1); s = co[2][t.long()].view(2, 1, 1, 1)
    g = (scaled * a + noise * s).to(torch.bfloat16).permute(0, 3, 1, 2).cpu()
    print("gpu torch == ref", torch.equal(g, ref), "gpu torch == ours", torch.equal(g, ours))
