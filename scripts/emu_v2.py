"""numpy/pure-Python emulator of the v2 blind-rotation kernel's index math (layouts A/B/C,
stream twiddles, Harvey butterflies, MAC, CRT).  Dev tool for kernel work; not the product."""
import numpy as np, sys
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
import oracle_ctypes as O
N=1024
Q=[134215681,134203393]
M32=0xFFFFFFFF
def powmod(b,e,q): return pow(b,e,q)
def brv(x,b=10): return int('{:0{w}b}'.format(x,w=b)[::-1],2)
tabs=[]
for s,q in enumerate(Q):
    psi=None
    for g in range(2,1000):
        c=pow(g,(q-1)//2048,q)
        if pow(c,1024,q)==q-1: psi=c;break
    ipsi=pow(psi,q-2,q)
    P=[pow(psi,brv(k),q) for k in range(N)]; IP=[pow(ipsi,brv(k),q) for k in range(N)]
    sh=lambda w: (w<<32)//q
    tabs.append(dict(psi=P,psip=[sh(w) for w in P],ipsi=IP,ipsip=[sh(w) for w in IP]))
# twiddle streams as in build_v2_twiddles
def streams(s):
    t=tabs[s]; tsf=[];tsi=[]
    for K in range(5,1,-1):
        for g in range(1<<(5-K)):
            tsf.append([(t['psi'][i],t['psip'][i]) for i in [(1<<(9-K))+((L>>2)<<(5-K))+g for L in range(64)]])
    for K in range(1,-1,-1):
        for g in range(1<<(3-K)):
            tsf.append([(t['psi'][i],t['psip'][i]) for i in [(1<<(9-K))+(L<<(3-K))+g for L in range(64)]])
    for K in range(0,4):
        for g in range(1<<(3-K)):
            tsi.append([(t['ipsi'][i],t['ipsip'][i]) for i in [(1<<(9-K))+(L<<(3-K))+g for L in range(64)]])
    for K in range(4,6):
        for g in range(1<<(5-K)):
            tsi.append([(t['ipsi'][i],t['ipsip'][i]) for i in [(1<<(9-K))+((L>>2)<<(5-K))+g for L in range(64)]])
    tuf=[(t['psi'][i],t['psip'][i]) for i in range(16)]; tui=[(t['ipsi'][i],t['ipsip'][i]) for i in range(16)]
    return tuf,tui,tsf,tsi
def umin(a,b): return a if a<b else b
def bf_ct(x,y,w,wp,q):
    q2=2*q
    u=x
    t=(y*w - ((y*wp)>>32)*q)&M32
    assert u+t < 2**32 and u+q2 < 2**32
    return (u+t)&M32, (u-t+q2)&M32
def bf_gs(x,y,w,wp,q):
    q2=2*q
    s=(x+y)&M32; t=(x-y+q2)&M32
    return umin(s,(s-q2)&M32), (t*w-((t*wp)>>32)*q)&M32
def jA(L,r): return L+64*r
def jB(L,r): return (L&3)|(r<<2)|((L>>2)<<6)
def jC(L,r): return 16*L+r
def relayout(x, src, dst):
    # x[L][r] in layout src -> layout dst
    vals={}
    for L in range(64):
        for r in range(16): vals[src(L,r)]=x[L][r]
    return [[vals[dst(L,r)] for r in range(16)] for L in range(64)]
def ntt_fwd(xs, s):
    q=Q[s]; tuf,tui,tsf,tsi=streams(s)
    for K in range(9,5,-1):
        d=1<<(K-6)
        for L in range(64):
            for r in range(16):
                if r&d: continue
                w,wp=tuf[(1<<(9-K))+(r>>(K-5))]
                for x in xs: x[L][r],x[L][r+d]=bf_ct(x[L][r],x[L][r+d],w,wp,q)
    xs=[relayout(x,jA,jB) for x in xs]
    slot=0
    for K in range(5,1,-1):
        d=1<<(K-2); cnt=1<<(5-K)
        for L in range(64):
            for r in range(16):
                if r&d: continue
                w,wp=tsf[slot+(r>>(K-1))][L]
                for x in xs: x[L][r],x[L][r+d]=bf_ct(x[L][r],x[L][r+d],w,wp,q)
        slot+=cnt
    xs=[relayout(x,jB,jC) for x in xs]
    for K in range(1,-1,-1):
        d=1<<K; cnt=1<<(3-K)
        for L in range(64):
            for r in range(16):
                if r&d: continue
                w,wp=tsf[slot+(r>>(K+1))][L]
                for x in xs: x[L][r],x[L][r+d]=bf_ct(x[L][r],x[L][r+d],w,wp,q)
        slot+=cnt
    return xs
# compare forward with oracle-style NTT
def ref_fwd(a,s):
    q=Q[s]; a=[v%q for v in a]; t=N; m=1; P=tabs[s]['psi']
    while m<N:
        t//=2
        for i in range(m):
            S=P[m+i]
            for j in range(2*i*t,2*i*t+t):
                U=a[j]; V=a[j+t]*S%q; a[j]=(U+V)%q; a[j+t]=(U-V)%q
        m*=2
    return a
def ntt_inv(xs,s):
    q=Q[s]; tuf,tui,tsf,tsi=streams(s)
    slot=0
    for K in range(0,4):
        d=1<<K; cnt=1<<(3-K)
        for L in range(64):
            for r in range(16):
                if r&d: continue
                w,wp=tsi[slot+(r>>(K+1))][L]
                for x in xs: x[L][r],x[L][r+d]=bf_gs(x[L][r],x[L][r+d],w,wp,q)
        slot+=cnt
    xs=[relayout(x,jC,jB) for x in xs]
    for K in range(4,6):
        d=1<<(K-2); cnt=1<<(5-K)
        for L in range(64):
            for r in range(16):
                if r&d: continue
                w,wp=tsi[slot+(r>>(K-1))][L]
                for x in xs: x[L][r],x[L][r+d]=bf_gs(x[L][r],x[L][r+d],w,wp,q)
        slot+=cnt
    xs=[relayout(x,jB,jA) for x in xs]
    for K in range(6,10):
        d=1<<(K-6)
        for L in range(64):
            for r in range(16):
                if r&d: continue
                w,wp=tui[(1<<(9-K))+(r>>(K-5))]
                for x in xs: x[L][r],x[L][r+d]=bf_gs(x[L][r],x[L][r+d],w,wp,q)
    return xs

def _selftest():
    rng=np.random.default_rng(0)
    a=[int(v) for v in rng.integers(0,Q[0],N)]
    x=[[a[jA(L,r)] for r in range(16)] for L in range(64)]
    out=ntt_fwd([x],0)[0]
    ref=ref_fwd(a,0)
    got=[None]*N
    for L in range(64):
        for r in range(16): got[jC(L,r)]=out[L][r]%Q[0]
    print('fwd ok', got==ref, sum(g!=r for g,r in zip(got,ref)))
    # inverse of forward: inv(fwd(a)) = N*a
    y=[[ref[jC(L,r)] for r in range(16)] for L in range(64)]
    back=ntt_inv([y],0)[0]
    ninv=pow(N,Q[0]-2,Q[0])
    got=[None]*N
    for L in range(64):
        for r in range(16): got[jA(L,r)]=back[L][r]*ninv%Q[0]
    print('inv ok', got==a)
    # ---- full cmux emulation vs oracle
    R32=1<<32
    def qinv_neg(q):
        inv=q
        for _ in range(5): inv=(inv*(2-q*inv))&M32
        return (-inv)&M32
    def crt(x0,x1):
        q0,q1=Q
        h=pow(q0%q1,q1-2,q1)
        x0r=x0-q1 if x0>=q1 else x0
        d=(x1-x0r)%q1
        t=d*h%q1
        X=x0+q0*t
        M=q0*q1
        if X>M//2: X-=M
        return X&M32
    bk=rng.integers(-2**31,2**31,(1,4,2,N),dtype=np.int64)   # one key index [i][p][c][N]
    bkntt={}
    for s in range(2):
        q=Q[s]; scale=pow(N,q-2,q)*(R32%q)%q
        for p in range(4):
            for c in range(2):
                bkntt[(s,p,c)]=[v*scale%q for v in ref_fwd([int(v) for v in bk[0,p,c]],s)]
    def cmux(acc,a):
        # acc: [2][N] uint32 ints
        O_all={}
        for s in range(2):
            q=Q[s]
            D=[]
            for c in range(2):
                d0=[[0]*16 for _ in range(64)]; d1=[[0]*16 for _ in range(64)]
                for L in range(64):
                    for r in range(16):
                        j=L+64*r; si=(j-a)&2047; v=acc[c][si&1023]; rot=(-v)&M32 if si&1024 else v
                        t=(rot-acc[c][j]+2149580800)&M32
                        d0[L][r]=((t>>22)&1023)+(q-512); d1[L][r]=((t>>12)&1023)+(q-512)
                D+= [d0,d1]
            D=ntt_fwd(D,s)
            qi=qinv_neg(q)
            O=[[[0]*16 for _ in range(64)] for _ in range(2)]
            for L in range(64):
                for r in range(16):
                    dd=[D[p][L][r] for p in range(4)]
                    j=16*L+r
                    for c in range(2):
                        x=sum(dd[p]*bkntt[(s,p,c)][j] for p in range(4))
                        m=(x&M32)*qi&M32
                        t=((x+m*q)>>32)&M32
                        O[c][L][r]=umin(t,(t-2*q)&M32)
            O=ntt_inv(O,s)
            for c in range(2):
                for L in range(64):
                    for r in range(16):
                        O[c][L][r]=umin(O[c][L][r],(O[c][L][r]-q)&M32)
            O_all[s]=O
        new=[[0]*N for _ in range(2)]
        for c in range(2):
            for L in range(64):
                for r in range(16):
                    j=L+64*r
                    new[c][j]=(acc[c][j]+crt(O_all[0][c][L][r],O_all[1][c][L][r]))&M32
        return new
    acc0=rng.integers(0,2**32,(2,N),dtype=np.int64)
    accl=[[int(v) for v in acc0[c]] for c in range(2)]
    a=77
    emu=cmux(accl,a)
    # oracle: key with bk index 0 = our bk; pad a full 500-key array with zeros
    fullbk=np.zeros((500,4,2,N),np.int32); fullbk[0]=bk[0].astype(np.int32)
    ok=O.OracleKey(fullbk,None,use_ntt=False)
    want=ok.mux_rotate(acc0.astype(np.uint32).view(np.int32) if False else (acc0.astype(np.int64)-( (acc0>=2**31)*2**32)).astype(np.int32),0,a)
    want=want.astype(np.int64)&M32
    print('cmux ok', all(emu[c][j]==want[c][j] for c in range(2) for j in range(N)))

if __name__ == "__main__":
    _selftest()
