import sys, torch
sys.path.insert(0, "/root/repo")
from fasttalk_llm_microservice_amd.ops import quant as Q
torch.manual_seed(0)
dev="cuda"
for n,k,splits,m in [(1024,512,1,17),(1024,1024,1,17),(1024,1536,1,17),(1024,2048,1,17),(1024,4096,4,17),(1024,4096,8,17),(1024,4096,4,64),(1024,1024,1,64)]:
    w=torch.randn(n,k)*0.05
    q,z,s=Q.quantize_w4(w)
    W=Q.pack_w4(q.to(dev),z.to(dev),s.to(dev))
    wdq=Q.dequantize_w4(q,z,s)
    x=torch.randn(m,k).bfloat16()
    ref=x.float()@wdq.t()
    if splits==1:
        out=torch.full((m,n),float("nan"),device=dev).bfloat16()
        y=Q.w4_gemm(x.to(dev),W,out=out,nt=1,xr=2).float().cpu()
    else:
        ws=torch.full((splits*m*n,),float("nan"),device=dev)
        Q.w4_gemm(x.to(dev),W,ws=ws,splits=splits,nt=1,xr=2)
        y=ws.view(splits,m,n).cpu()
        bad_split=[int(torch.isnan(y[i]).sum()) for i in range(splits)]
        y=y.sum(0)
        print("  nan per split", bad_split)
    err=(y-ref).abs()
    badr=(err>0.05*ref.abs().max()).any(1).nonzero().flatten().tolist()
    badc=(err>0.05*ref.abs().max()).any(0).nonzero().flatten().tolist()
    print(n,k,splits,m,"nch",k//splits//512,"maxerr",float(err.nan_to_num(1e9).max()),"badrows",badr[:10],len(badr),"badcols",badc[:8],len(badc),flush=True)
