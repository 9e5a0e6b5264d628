rule rootlist {
 strings:
  $r = /.{2,3}/
  $s = "abc"
 condition: $r and $s
}
