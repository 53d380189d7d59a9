"""Static count of serialised loads per kernel: a `global_load`/`buffer_load` followed by an
`s_waitcnt vmcnt(0)` before the next load (the load's latency is paid alone). Used to find loads
that the compiler sank into branches (one wait per conditional load).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -I aa-admm_amd/csrc --cuda-device-only -S -o k.s FILE.hip
    python tools/isa_serial.py FILTER k.s [k2.s ...]
"""
import re,subprocess,sys
def kernels(path):
    s=open(path).read().split('\n'); cur=None; out={}
    for l in s:
        m=re.match(r'^(_Z\S+):', l)
        if m: cur=m.group(1); out[cur]=[]; continue
        if cur is not None:
            if l.startswith('.Lfunc_end'): cur=None; continue
            out[cur].append(l.strip())
    return out
def stats(body):
    loads=sum(1 for l in body if re.match(r'(global|buffer)_load',l))
    ser=0; pend=False
    for l in body:
        if re.match(r'(global|buffer)_load',l): pend=True
        elif re.match(r's_waitcnt.*vmcnt\(0\)',l) and pend: ser+=1; pend=False
    return loads, ser
if __name__=="__main__":
    filt=sys.argv[1]
    for path in sys.argv[2:]:
        for k,body in kernels(path).items():
            if filt not in k: continue
            l,s_=stats(body)
            name=subprocess.run(['c++filt',k],capture_output=True,text=True).stdout.strip()
            print(f"{path[-8:]} {name[:70]:70s} loads {l:4d} serial {s_:4d}")
