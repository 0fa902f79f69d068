"""Forward outputs of two builds of the library on the same inputs (bit-for-bit check).
usage: python tools/cmp_libs.py <libA> <libB>   ('' = the in-tree library)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [("n", "bf16", 4, 640), ("s", "fp16", 2, 320), ("n", "fp16", 2, 224), ("m", "bf16", 2, 480)]


def child(out):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "yolo-infer-pt_amd"))
    import torch
    from yolo_hip import synth
    from yolo_hip.engine import Engine
    from nets import nn
    res = {}
    for v, dt, b, sz in CASES:
        dtype = torch.bfloat16 if dt == "bf16" else torch.float16
        torch.manual_seed(0)
        model = getattr(nn, f"yolo_v11_{v}")(80)
        model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
        model.eval()
        dev = torch.device("cuda", 0)
        eng = Engine(*model._yh_arch, dev, dtype)
        eng.load_module(model)
        x = synth.synth_scenes(b, sz, sz, seed=34).to(dev, dtype)
        y = eng.forward(x)
        torch.cuda.synchronize()
        res[f"{v}_{dt}_{b}_{sz}"] = y.cpu()
    torch.save(res, out)


def main():
    if sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    import torch
    outs = []
    for k, lib in enumerate(sys.argv[1:3]):
        env = dict(os.environ)
        env.pop("YH_LIB", None)
        if lib:
            env["YH_LIB"] = lib
        out = os.path.join(ROOT, "gpurun_out", f"cmp_{k}.pt")
        subprocess.run([sys.executable, __file__, "--child", out], env=env, check=True, timeout=600)
        outs.append(torch.load(out, weights_only=True))
    bad = 0
    for key in outs[0]:
        a, b = outs[0][key], outs[1][key]
        same = torch.equal(a, b)
        bad += not same
        print(key, "bit-identical" if same else f"DIFFER max {(a.float() - b.float()).abs().max().item()}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
