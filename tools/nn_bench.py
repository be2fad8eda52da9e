"""Leaf-eval net variants at the self-play batch (256 x 8 x 20 x 20): time per forward and the
max deviation of p/v from the fp32 eval-mode ResNet. Run on a GPU box."""
import sys, os, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from blokus_rl_amd.nets import ResNet, FusedResNet, LeafResNet

torch.manual_seed(0)
dev = "cuda"
net = ResNet(20, 4, 30433, 5).to(dev).eval()
# non-trivial BN statistics
with torch.no_grad():
    for m in net.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.2, 0.2); m.running_var.uniform_(0.5, 1.5)
            m.weight.uniform_(0.8, 1.2); m.bias.uniform_(-0.1, 0.1)
x = (torch.rand(256, 8, 20, 20, device=dev) < 0.3).float()
with torch.inference_mode():
    ref_p, ref_v = net(x)

def timeit(fn, n=30):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / n

res = {}
def run(name, model, dtype=None, cl=False, graph=True):
    xx = x.contiguous(memory_format=torch.channels_last) if cl else x
    if cl: model = model.to(memory_format=torch.channels_last)
    def fwd():
        with torch.inference_mode():
            if dtype is None:
                return model(xx)
            with torch.autocast("cuda", dtype=dtype):
                return model(xx)
    out = fwd()
    if graph:
        s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fwd(); fwd()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = fwd()
        ms = timeit(g.replay)
    else:
        ms = timeit(fwd)
    p, v = out
    dp = (p.float().exp() - ref_p.exp()).abs().max().item()
    dlp = (p.float() - ref_p).abs().max().item()
    dv = (v.float() - ref_v).abs().max().item()
    res[name] = {"ms": ms, "max_abs_dp": dp, "max_abs_dlogp": dlp, "max_abs_dv": dv}
    print(name, json.dumps(res[name]), flush=True)

run("resnet_fp32_eager", net, graph=False)
run("resnet_fp32_graph", net)
fused = FusedResNet(net).eval()
run("fused_fp32", fused)
run("leaf_fp32_cl", LeafResNet(net).eval(), None, cl=True)
run("leaf_fp32_cl_graph", LeafResNet(net).eval(), None, cl=True, graph=True)
torch.backends.cudnn.benchmark = True
run("fused_fp32_bench", fused)
run("fused_fp16", fused, torch.float16)
run("fused_bf16", fused, torch.bfloat16)
run("fused_fp16_cl", FusedResNet(net).eval(), torch.float16, cl=True)
run("fused_bf16_cl", FusedResNet(net).eval(), torch.bfloat16, cl=True)
run("fused_fp32_cl", FusedResNet(net).eval(), None, cl=True)
json.dump(res, open("gpurun_out/nn_bench.json", "w"), indent=1)
