include "../baz.yar"

rule bar { condition: baz }
