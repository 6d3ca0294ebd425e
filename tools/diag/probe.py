import ctypes, os
here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "probe.so"))
tr = (ctypes.c_int * 256)(); mf = (ctypes.c_float * 1024)()
print("rc", lib.run_probes(tr, mf))
print("TR: lane -> [(row,col)]x4")
for l in range(64):
    print(l, [(tr[l*4+e] // 64, tr[l*4+e] % 64) for e in range(4)])
print("MFMA32: lane -> rows of col (value//32 = k/row, value%32 = col)")
for l in (0, 1, 31, 32, 33, 63):
    print(l, [(int(mf[l*16+e]) // 32, int(mf[l*16+e]) % 32) for e in range(16)])
