rule hex_jumps {
 strings:
  $a = { 4D 5A ?? ?? 50 45 [2-6] 11 22 }
  $b = { AA BB CC DD [1-3] EE [0-2] FF 01 }
  $c = { 10 20 [4] 30 40 50 60 }
  $d = { 71 72 73 74 ?5 7? [1-10] 75 }
  $e = { 01 02 ~03 04 05 06 }
  $f = { 81 82 83 84 [1-2] 85 [1-2] 86 [1-2] 87 }
 condition: any of them
}
rule hex_prefix {
 strings:
  $a = { 9A 9B [1-4] C1 C2 C3 C4 }
  $b = { E1 ?? E3 [2-3] F1 F2 F3 F4 F5 }
  $c = { 5? 6? 7? 8? 91 92 93 94 }
 condition: any of them
}
rule hex_long_jump {
 strings:
  $a = { 31 41 59 26 [100-3000] 53 58 97 93 }
 condition: $a
}
