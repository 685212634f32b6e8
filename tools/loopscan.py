import re,sys
S=open(sys.argv[1]).read().split('\n')
cur=None; funcs={}
for i,l in enumerate(S):
    m=re.match(r'^(_Z\w+):',l)
    if m: cur=m.group(1); funcs[cur]=[]
    if cur: funcs[cur].append(l)
for f,L in funcs.items():
    if sys.argv[2] not in f: continue
    # find loop header and backedge
    hdr=[i for i,l in enumerate(L) if 'Loop Header' in l]
    for h in hdr:
        lab=L[h].split(':')[0]
        be=[i for i,l in enumerate(L) if re.search(r's_cbranch\w* '+re.escape(lab)+r'$',l)]
        if not be: continue
        body=L[h:be[-1]+1]
        sc=sum('scratch_' in l for l in body); vm0=sum('vmcnt(0)' in l for l in body)
        print(f[:60], 'loop', lab, 'lines', len(body), 'scratch', sc, 'vmcnt0', vm0, 'mfma', sum('v_mfma' in l for l in body))
