import sys; sys.path.insert(0,'.')
import deneva_amd as d, torch
b=d.gen_ycsb(n_txn=1<<20, zipf_theta=0.9)
db=b.to_torch('cuda:0')
with d.Engine(0) as e:
    for _ in range(2): rc,_,st=e.occ_validate_epoch(db)
    print(st['device_ms'], st['rounds'])
