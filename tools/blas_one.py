import sys, torch
M, N, K = (int(x) for x in sys.argv[1:4])
a = torch.randn(M, K, device="cuda").bfloat16(); w = torch.randn(N, K, device="cuda").bfloat16()
for _ in range(5): torch.matmul(a, w.t())
torch.cuda.synchronize()
