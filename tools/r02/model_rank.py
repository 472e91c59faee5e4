import sys; sys.path.insert(0,'/root/repo')
import pconv
n=pconv.native
for (ch,rows,rb,steps) in [("grey",32768,32768,8),("grey",32768,32768,6),("rgb",2520,5760,8),("rgb",8192,24576,8),("rgb",395,5760,8)]:
    t=n.swar_model_table(steps, ch, rows, rb)
    t.sort(key=lambda r:r[6])
    print(ch, rows, rb, steps, [(f"{r[0]},{r[1]},{r[2]}", r[3], round(r[6]/1e3)) for r in t[:8]])
