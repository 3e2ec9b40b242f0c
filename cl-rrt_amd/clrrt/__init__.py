"""clrrt — host-side Python binding of libclrrt (the MI355X closed-loop RRT engine)."""
