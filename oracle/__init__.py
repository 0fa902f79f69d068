"""CPU oracle of the YOLOv11 inference path — TEST INFRASTRUCTURE ONLY.

This package restates the reference algorithm (t0saki/YOLO-Infer-pt) on the CPU
so the HIP kernels can be checked against it at any seed, size and variant:

  oracle.forward  eval forward of nets/nn.py:8-347 + utils/util.py:85-96 as plain
                  functional torch-CPU ops on a state_dict, in float32 or float64
  oracle.nms      utils/util.py:123-169 + the torchvision.ops.nms contract in numpy

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
it, and only as the checker (or the timed CPU baseline). The product path
(nets.nn / utils.util / yolo_hip) never imports it.

Pinning: the restatement is checked against golden vectors produced by the
reference's own Python (imported in the survey/build container with a stub
`torchvision` module, see oracle/make_goldens.py) and committed under
tests/golden/. torchvision is absent from the container, so the NMS kernel
contract itself (greedy, IoU > thr, area without +1) is a restatement of
torchvision's documented behaviour: "parity unpinned" for that single
third-party piece; the reference's own candidate selection, ordering,
class offsets and truncation around it are pinned by the goldens.
"""
