"""Saves one v11_x bf16 1280 b16 head output (scene seed 300) made by the shipped library to /tmp/y_c5.pt,
for tools/nms_trace.py (YH_NMS_Y=/tmp/y_c5.pt) under the diagnostic build."""
import sys, torch
sys.path.insert(0, "."); sys.path.insert(0, "yolo-infer-pt_amd")
from nets import nn
from yolo_hip import synth
from yolo_hip.engine import Engine
torch.manual_seed(0)
m = nn.yolo_v11_x(80); m.load_state_dict(synth.synth_state_dict(m.state_dict(), seed=0)); m.eval()
dev = torch.device("cuda", 0)
e = Engine(*m._yh_arch, dev, torch.bfloat16); e.load_module(m)
y = e.forward(synth.synth_scenes(16, 1280, 1280, seed=300).to(dev, torch.bfloat16))
torch.save(y.cpu(), "/tmp/y_c5.pt")
print("saved", tuple(y.shape))
