rule bytekeys {
 strings:
  $a = { 00 }
  $b = "Q"
  $c = { FF }
  $d = "abc"
  $e = "wxyz"
  $f = { 00 00 41 }
  $g = "Qrst"
 condition: any of them
}
