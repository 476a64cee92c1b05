import sys
p=sys.argv[1]; s=open(p).read()
old="""        _Pragma("unroll") for (int kk = 0; kk < QMC_KMAX; ++kk)                              \\
          if (kk < K && (unsigned)(gr[kk] >> 32) != tag)                                     \\
            gr[kk] = __hip_atomic_load(slot + (int64_t)kk * MC_SLOT + gi, __ATOMIC_RELAXED,  \\
                                       __HIP_MEMORY_SCOPE_AGENT);                            \\"""
new="""        _Pragma("unroll") for (int kk = 0; kk < QMC_KMAX; ++kk)                              \\
          if (kk < K && __any((unsigned)(gr[kk] >> 32) != tag))                              \\
            gr[kk] = __hip_atomic_load(slot + (int64_t)kk * MC_SLOT + gi, __ATOMIC_RELAXED,  \\
                                       __HIP_MEMORY_SCOPE_AGENT);                            \\"""
assert s.count(old)==1; s=s.replace(old,new); open(p,'w').write(s)
