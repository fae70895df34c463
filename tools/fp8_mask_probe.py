"""fp8 layer-set accuracy probe: one ControlLDM forward at B = 2 with fp8 operands on the
layers of each TAIR_FP8_OPS mask vs the fp32 oracle; prints v rel-L2 per mask.  Each mask runs in a fresh
child process (the mask is read once per process, at model creation).

    python tools/fp8_mask_probe.py 0 1 2 4 8 16 31
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(mask):
    sys.path.insert(0, ROOT)
    import torch
    from oracle.ldm_ref import ControlLDMRef
    from tair_amd.cldm import ControlLDM
    from tair_amd.weights import manifest, perturb_norms, synthetic_state_dict
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    sd = perturb_norms(synthetic_state_dict(manifest(), seed=0))
    m = ControlLDM(max_batch=2, with_vae=False, fp8=mask != 0)
    m.load_state_dict(sd)
    ref = ControlLDMRef().cuda().eval()
    ref.load_state_dict(sd, strict=True)
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, 4, 64, 64, generator=g).cuda()
    c_img = torch.randn(2, 4, 64, 64, generator=g).cuda()
    c_txt = torch.randn(1, 77, 1024, generator=g).cuda()
    t = torch.tensor([999, 487], device="cuda")
    with torch.no_grad():
        v, _ = m(x, t, {"c_txt": c_txt, "c_img": c_img})
        rv, _ = ref(x, t, {"c_txt": c_txt.expand(2, -1, -1), "c_img": c_img})
    e = ((v.double() - rv.double()).norm() / rv.double().norm()).item()
    print(json.dumps({"mask": mask, "rel_l2_v": e}), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--one":
        one(int(sys.argv[2]))
        sys.exit(0)
    for mk in sys.argv[1:]:
        env = dict(os.environ, TAIR_FP8_OPS=mk)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--one", mk], env=env, timeout=300)
        if r.returncode:
            sys.exit(r.returncode)
