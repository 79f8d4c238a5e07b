"""One trial of a rocprofv3 rocpd database (kernels of every queue by start time:
offset, duration, idle gap, queue) from one k_reduce to the next. usage:
python scripts/trial_timeline.py run_results.db [k = k_reduce index, default -6]"""
import sqlite3,sys
db=sqlite3.connect(sys.argv[1])
rows=db.execute("select name,start,end,queue_id from kernels order by start").fetchall()
idx=[i for i,r in enumerate(rows) if 'k_reduce(' in r[0]]
k=int(sys.argv[2]) if len(sys.argv)>2 else -6
a,b=idx[k],idx[k+1]
t0=rows[a][1];busy=t0
for r in rows[a:b+1]:
    s,e=r[1],r[2]
    nm=r[0].split('(')[0].replace('sqlm::','').replace('void ','')[:45]
    print(f"{(s-t0)/1000:8.2f} {(e-s)/1000:7.2f} gap {(s-busy)/1000:6.2f} q{r[3]} {nm}")
    busy=max(busy,e)
