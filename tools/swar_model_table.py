import sys; sys.path.insert(0,'.')
import torch, pconv
n=pconv.native
n.set_device(0)
for (st,ch,rows,rb) in [(8,'grey',32768,32768),(8,'rgb',8192,24576),(8,'rgb',2520,5760)]:
    t=n.swar_model_table(st,ch,rows,rb)
    print(st,ch,rows,rb)
    for r in sorted(t,key=lambda r:r[-1]): print("  ",r)
