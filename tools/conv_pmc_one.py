import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from flexflow_train_amd import kernels as K
N, H, C, Ko, R = 256, 14, 256, 256, 3
x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
w = (torch.randn(Ko, R, R, C, device="cuda") * 0.05).to(torch.bfloat16).contiguous()
y = K.conv2d_fwd(x, w, None, (1, 1), (1, 1))
dy = torch.randn_like(y).contiguous(memory_format=torch.channels_last)
dw = torch.zeros(Ko * R * R * C, device="cuda")
for _ in range(5):
    K.conv2d_fwd(x, w, None, (1, 1), (1, 1))
    K.conv2d_dgrad(dy, w, tuple(x.shape), (1, 1), (1, 1))
    K.conv2d_wgrad(x, dy, dw, R, R, (1, 1), (1, 1))
torch.cuda.synchronize()
print("done")
