import ctypes as C, time, sys, os
R=os.environ.get('GRAFT_REPO_ROOT','/root/repo')
sys.path.insert(0,R); sys.path.insert(0,R+'/tests/golden'); sys.path.insert(0,R+'/tests')
import inputs as I
import libapenetwork_amd as amd
from lz4util import buf
L=amd.lib(); orc=C.CDLL(R+'/oracle/liblz4_oracle.so'); ref=C.CDLL(R+'/oracle/_ref/libape_lz4_ref.so')
st=C.create_string_buffer(16416)
L.hst_compress_extstate.argtypes=[C.c_void_p]*3+[C.c_int]*3
def clock(fn,reps=400):
    for _ in range(20): fn()
    best=1e9
    for k in range(5):
        t0=time.perf_counter()
        for _ in range(reps): fn()
        best=min(best,(time.perf_counter()-t0)/reps*1e6)
    return best
for n in (1024,8192,65536):
    s=I.make("comp",n,seed=5); b=buf(s); bound=amd.compressBound(n); o=C.create_string_buffer(bound+64)
    r=L.APE_LZ4_compress_default(b,o,n,bound); cb=buf(o.raw[:r]); d=C.create_string_buffer(n+64)
    res={}
    for name,fn in (("prod_c",lambda: L.APE_LZ4_compress_default(b,o,n,bound)),("hst_c",lambda: L.hst_compress_extstate(st,b,o,n,bound,1)),("orc_c",lambda: orc.orc_compress_default(b,o,n,bound)),("ref_c",lambda: ref.APE_LZ4_compress_default(b,o,n,bound)),
                    ("prod_d",lambda: L.APE_LZ4_decompress_safe(cb,d,r,n)),("orc_d",lambda: orc.orc_decompress_safe(cb,d,r,n)),("ref_d",lambda: ref.APE_LZ4_decompress_safe(cb,d,r,n))):
        res[name]=clock(fn)
    print(n, " ".join("%s %.2f"%(k,v) for k,v in res.items()))
