cd $GRAFT_REPO_ROOT
export APE_LZ4_LIB=$PWD/libapenetwork_amd/libape_lz4_amd_dbg.so
timeout -k 10 120 python3 tools/kernel_driver.py 64 1 2>&1 | grep -v amdgpu.ids | head -20
timeout -k 10 120 python3 - <<'PY' 2>&1 | grep -v amdgpu.ids | head -20
import sys; sys.path.insert(0,'.')
import torch, libapenetwork_amd as amd
n=65536
for name, data in [("zeros", torch.zeros((2,n),dtype=torch.uint8)), ("text", torch.tensor(bytearray((b"the quick brown fox jumps over the lazy dog " * 4000)[:2*n]),dtype=torch.uint8).view(2,n))]:
    src=data.cuda(); sizes=torch.full((2,),n,dtype=torch.int32,device='cuda')
    slot=(amd.compressBound(n)+15)//16*16
    comp=torch.zeros((2,slot),dtype=torch.uint8,device='cuda'); csz=torch.zeros(2,dtype=torch.int32,device='cuda')
    amd.compress_batch(src,sizes,comp,csz); torch.cuda.synchronize(); print(name, csz.tolist())
PY
