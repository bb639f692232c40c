import random
MC=[17, 15, 41, 16, 2, 28, 13, 13, 39, 18, 34, 20]
M64=(1<<64)-1
def mds_ref(s): return [sum(MC[(y-x)%12]*s[y] for y in range(12)) for x in range(12)]
def circ_fft(v):  # v: 12 ints; wrapping 64-bit arithmetic
    u0=[0]*3;u1=[0]*3;p=[0]*3;q=[0]*3
    for b in range(3):
        S=[v[(9*a+4*b)%12] for a in range(4)]
        t0=S[0]+S[2]; t1=S[1]+S[3]
        u0[b]=(t0+t1)&M64; u1[b]=(t0-t1)&M64; p[b]=(S[0]-S[2])&M64; q[b]=(S[1]-S[3])&M64
    s0=(u0[0]+u0[1]+u0[2])&M64
    w=[0]*12
    for b in range(3):
        b1=(b+2)%3; b2=(b+1)%3
        V0=((s0+u0[b1])<<4)&M64
        V1=(-u1[b]+8*u1[b1]+2*u1[b2])&M64
        re=(2*p[b]+q[b]-p[b1]+4*q[b1]-16*p[b2]+q[b2])&M64
        im=(2*q[b]-p[b]-q[b1]-4*p[b1]-16*q[b2]-p[b2])&M64
        A=(V0+V1)&M64; B=(V0-V1)&M64
        w[(0+4*b)%12]=(A+re)&M64; w[(18+4*b)%12]=(A-re)&M64
        w[(9+4*b)%12]=(B+im)&M64; w[(27+4*b)%12]=(B-im)&M64
    return w
for _ in range(2000):
    v=[random.randrange(2**32) for _ in range(12)]
    assert circ_fft(v)==mds_ref(v), (v)
print("ok")
