import torch
x=torch.empty(16*256*256*64,device="cuda"); y=torch.empty_like(x)
def t(f,n=20):
    f(); torch.cuda.synchronize()
    e0,e1=torch.cuda.Event(True),torch.cuda.Event(True); e0.record()
    for _ in range(n): f()
    e1.record(); torch.cuda.synchronize(); return e0.elapsed_time(e1)/n
for _ in range(3):
    a=t(lambda: x.fill_(1.0)); b=t(lambda: y.copy_(x)); c=t(lambda: x.sum())
    print(f"fill {a*1e3:.1f}us {x.numel()*4/a/1e9:.2f}TB/s  copy {b*1e3:.1f}us {2*x.numel()*4/b/1e9:.2f}TB/s  sum {c*1e3:.1f}us {x.numel()*4/c/1e9:.2f}TB/s")
