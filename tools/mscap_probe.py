import torch
dev = torch.device("cuda", 0)
x = torch.zeros(1 << 20, device=dev); y = torch.zeros(1 << 20, device=dev)
g = torch.cuda.CUDAGraph()
cap = torch.cuda.Stream(dev)
cap.wait_stream(torch.cuda.current_stream(dev))
with torch.cuda.graph(g, stream=cap):
    cs = torch.cuda.current_stream(dev)
    se, sd = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    se.wait_stream(cs); sd.wait_stream(cs)
    done = []
    for k in range(20):
        if k >= 2:
            se.wait_event(done[k - 2])
        with torch.cuda.stream(se):
            x.add_(1)
        e = torch.cuda.Event(); e.record(se); sd.wait_event(e)
        with torch.cuda.stream(sd):
            y.add_(x)
        d = torch.cuda.Event(); d.record(sd); done.append(d)
    cs.wait_stream(se); cs.wait_stream(sd)
torch.cuda.synchronize()
g.replay(); torch.cuda.synchronize()
print("torch multistream capture ok", float(x[0]), float(y[0]))
