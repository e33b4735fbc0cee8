# volpath register-budget sweep: swap the library variant, time config 4
L=mitsuba3-nasa_amd/mitsuba_hip
cp $L/libmitsuba_hip.so /tmp/base.so
for w in base w3 w4; do
  if [ $w != base ]; then cp $L/libmitsuba_hip_$w.so $L/libmitsuba_hip.so; else cp /tmp/base.so $L/libmitsuba_hip.so; fi
  echo "$w: $(timeout -k 10 200 python tools/bench_volpath.py --no-cpu --steps 2 --grid 128 2>/dev/null | grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*' | tr '\n' ' ')"
done
cp /tmp/base.so $L/libmitsuba_hip.so
