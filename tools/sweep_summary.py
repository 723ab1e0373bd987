import json,sys
for c in sys.argv[1:]:
    s=open(f"gpurun_out/{c}.log").read()
    try: d=json.loads(s[s.index("{"):])
    except Exception as e: print(c, "FAILED", s[-2000:]); continue
    for k,v in d["ms(median,min)"].items():
        print(c,k,"vol %.4f total %.4f bdy %.4f hint %.4f steps %.3f"%(v["vol"][0],v["total"][0],v["bdy"][0],v["hint"][0],v["stepav"]), v.get("mismatches"))
