import sys, time, json
sys.path.insert(0, '.')
import torch
from pytorch_dppo_amd.config import dppo_preset
from pytorch_dppo_amd.parallel.dist import DistContext
from pytorch_dppo_amd.runtime.worker import DPPOWorker
dev = torch.device("cuda", 0)
p = dppo_preset(device="gpu", env_name="Humanoid-v2", num_envs=4096, exploration_size=65536, batch_size=65536, num_epoch=10, dtype="bf16")
w = DPPOWorker(p, DistContext(device=dev))
for i in range(3): w.iteration_step(defer=True)
torch.cuda.synchronize()
hs = []
t_all = time.perf_counter()
for i in range(10):
    t0 = time.perf_counter(); w.iteration_step(defer=True); hs.append(time.perf_counter() - t0)
torch.cuda.synchronize()
tot = time.perf_counter() - t_all
# pure host cost of the enqueue: time the launch calls of one epoch in isolation
eng = w.engine
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    eng.grad(None)
t_grad = (time.perf_counter() - t0) / 20
t0 = time.perf_counter()
for _ in range(20):
    eng.apply()
t_apply = (time.perf_counter() - t0) / 20
torch.cuda.synchronize()
print(json.dumps({"host_ms_per_iter(step call)": [round(h*1e3, 3) for h in hs], "wall_ms_per_iter": tot/10*1e3,
                  "host_us_grad_call": t_grad*1e6, "host_us_apply_call": t_apply*1e6}))
