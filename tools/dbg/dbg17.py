import sys; sys.path.insert(0, '.')
from tests.small import random_corpus
from oracle import oracle as O
from nemo_amd import engine as E
import numpy as np
c,_ = random_corpus(17, max_nodes=16)
s,f = c.success_iters(), c.failed_iters()
r = O.analyze(c, s, f)
e = E.Engine(0)
res = E.analyze(c, s, f, engine=e)
print("oracle", r.diff_mask.tolist(), r.missing.tolist())
print("gpu   ", res.diff_mask.tolist(), res.missing.tolist())
print("flags eq", np.array_equal(res.flags, r.flags))
g0 = 1
n0 = int(c.node_off[g0]); V = c.graph_size(g0)
topo = e.debug_copy("topo", 4*n0, 4*V).view(np.uint32)
nlev = e.debug_copy("nlev", 4*g0, 4).view(np.uint32)[0]
lvl = e.debug_copy("lvl", 4*(n0+g0), 4*(nlev+1)).view(np.uint32)
db = e.debug_copy("dbits", 0, V)
r0lab = e.debug_copy("r0lab", 0, 4*7).view(np.uint32)
print("topo", topo, "lvl", lvl, "dbits", [hex(x) for x in db])
print("r0lab", r0lab, "labels g0", c.label[n0:n0+V], "src labels", c.label[int(c.node_off[3]):int(c.node_off[4])])
