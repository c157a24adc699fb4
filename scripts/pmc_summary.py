import csv, sys, collections, re
def short(n):
    if 'gemm_xd' in n:
        m=re.search(r'XdCfg<([^>]*)>\s*,\s*(\d+)', n)
        return 'xd<%s> epi %s' % (m.group(1), m.group(2)) if m else 'xd'
    if 'gemm_w4' in n:
        m=re.search(r'gemm_w4_kernel<(\d+), (\d+)>', n)
        return 'w4 epi %s v%s' % m.groups() if m else 'w4'
    if 'gemm_ring' in n: return 'ring'
    if 'ingest_kernel' in n:
        m=re.search(r'ingest_kernel<(\d+), (\d+), (\d+), (\d+)>', n)
        return 'ingest S%s W%s %sx%s' % m.groups() if m else n[:40]
    if 'paged_decode_persist' in n: return 'decode_attn_persist'
    if 'Cijk' in n: return 'lib:'+n[:40]
    return n[:30]
agg=collections.defaultdict(lambda: collections.defaultdict(float)); cnt=collections.Counter()
for d in sys.argv[1:]:
    for r in csv.DictReader(open(d)):
        k=short(r['Kernel_Name'])
        agg[k][r['Counter_Name']]+=float(r['Counter_Value'])
        cnt[(k,r['Counter_Name'])]+=1
for k,v in agg.items():
    n=max(c for (kk,_),c in cnt.items() if kk==k)
    print(k, 'dispatches', n, {c: round(x/cnt[(k,c)],1) for c,x in v.items()})
