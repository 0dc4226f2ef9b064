import csv,glob,sys
f=glob.glob('/tmp/rw_prof/**/*kernel_trace.csv',recursive=True)
rows=list(csv.DictReader(open(f[0])))
out=open(sys.argv[1],'w')
for r in rows:
    if "k_lf" in r["Kernel_Name"] or "k_decode" in r["Kernel_Name"]: out.write('%s %s %.2f\n'%(r['Dispatch_Id'], r['Kernel_Name'][:70], (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3))
