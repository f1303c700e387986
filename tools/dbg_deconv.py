import sys, torch, numpy as np, torch.nn.functional as F
sys.path.insert(0, '.')
from image_denoising_amd import _lib
DEV='cuda'
def nhwc(t): return t.permute(0,2,3,1).contiguous()
for (N,H,W) in [(2,8,8),(3,13,37),(1,1,17),(1,2,16),(1,1,32),(2,3,40)]:
    torch.manual_seed(0)
    x=torch.randn(N,96,H,W,dtype=torch.float64); w=torch.randn(96,96,2,2,dtype=torch.float64)*0.1; b=torch.randn(96,dtype=torch.float64)*0.1
    ref=F.conv_transpose2d(x,w,b,stride=2)
    stride,off=104,4
    xg=nhwc(x.float()).to(DEV); wg,bg=w.float().to(DEV),b.float().to(DEV)
    pk=_lib.scratch(_lib.lib().dn_deconv2x2_x6_pack_size(),DEV)
    yg=torch.full((N,2*H,2*W,stride),7.0,device=DEV)
    _lib.call("dn_deconv2x2_forward_x6",xg.data_ptr(),N,H,W,wg.data_ptr(),bg.data_ptr(),yg.data_ptr(),stride,off,pk.data_ptr(),pk.numel(),torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    y=yg[...,off:off+96].permute(0,3,1,2).cpu().double()
    err=(y-ref).abs()
    bad=torch.nonzero(err>1e-4)
    print(N,H,W,'bad',bad.shape[0],'of',err.numel(), 'untouched7', int((y==7.0).sum()))
    if bad.shape[0]:
        px=set((int(a),int(c),int(d)) for a,_,c,d in bad.tolist())
        print('  bad pixels (n,Y,X) sample', sorted(px)[:12], 'count', len(px))
        chans=sorted(set(int(c) for _,c,_,_ in bad.tolist()))
        print('  channels', chans[:20], len(chans))
