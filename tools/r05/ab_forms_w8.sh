for c in D64 C5 16,12,2048,2048,64 4,12,4096,4096,64; do bash tools/r05/impl_ab.sh $c "prod:asm4p w8sfp:asm8 prod:auto" ; done
