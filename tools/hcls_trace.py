import os, sys, torch
sys.path[:0]=['.', 'yolo-infer-pt_amd']
os.environ['YH_HCLS_TRACE']='1'
from yolo_hip import synth
from yolo_hip.engine import Engine
from nets import nn
torch.manual_seed(0)
m=nn.yolo_v11_n(80); m.load_state_dict(synth.synth_state_dict(m.state_dict(), seed=0)); m.eval()
dev=torch.device('cuda',0)
e=Engine(*m._yh_arch, dev, torch.bfloat16); e.load_module(m)
x=synth.synth_scenes(32,640,640,seed=3).to(dev,torch.bfloat16)
e.set_graph(False)
for _ in range(3): y=e.forward(x)
torch.cuda.synchronize()
