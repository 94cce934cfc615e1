import torch, time, statistics
from kafka_llm_service_amd import ops
dev=torch.device("cuda:0")
B,V=64,128256
lg=torch.randn(B,V,device=dev).to(torch.bfloat16)
t=torch.full((B,),0.7,device=dev); tp=torch.ones(B,device=dev); tk=torch.zeros(B,dtype=torch.int32,device=dev)
sd=torch.arange(B,dtype=torch.int64,device=dev)
res=[]
for r in range(5):
    s,e=torch.cuda.Event(enable_timing=True),torch.cuda.Event(enable_timing=True)
    ops.sample(lg,t,tp,tk,sd); torch.cuda.synchronize(); s.record()
    for i in range(50): ops.sample(lg,t,tp,tk,sd)
    e.record(); torch.cuda.synchronize(); res.append(s.elapsed_time(e)*1e3/50)
print("sample 64x128256 bf16 T=0.7 us/call", round(statistics.median(res),1))
